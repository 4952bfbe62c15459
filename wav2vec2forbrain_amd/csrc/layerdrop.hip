// LayerDrop inside a captured (graph-replayed) training step.
//
// The reference skips an encoder layer when a host draw torch.rand([]) < layerdrop (TF w2v
// Wav2Vec2Encoder.forward, TF conf Wav2Vec2ConformerEncoder.forward). A captured HIP graph fixes
// its host-side control flow, so in a graph every layer is captured and the skip decision moves to
// the device: keep = hash(seed + epoch * phi, 0) >= thr(p), the same counter-based draw the
// dropout masks use (common.h), re-drawn on every replay because the step counter advances.
//   forward : out = keep ? layer_out : layer_in            (+ the bf16 copy of out)
//   backward: d_layer_out = keep ? dout : 0 ; d_layer_in = keep ? 0 : dout
// A skipped layer therefore contributes exact zeros to every weight gradient and passes its
// input gradient through unchanged, which is what skipping it does in the reference.
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {

__host__ __device__ inline uint32_t ld_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// identical to b2p_hash(seed, 0) / b2p_seed_eff (common.h), callable on the host for the query
__host__ __device__ inline bool ld_keep(uint64_t seed, uint64_t epoch, int has_epoch, uint32_t thr) {
  if (has_epoch) seed += 0x9E3779B97F4A7C15ull * epoch;
  const uint32_t k = (uint32_t)seed ^ ld_mix32((uint32_t)(seed >> 32) + 0x9E3779B9u);
  const uint32_t h = ld_mix32(ld_mix32(k) + k);
  return h >= thr;
}

__device__ __forceinline__ bool dev_keep(uint64_t seed, const uint64_t* epoch, uint32_t thr) {
  return epoch ? ld_keep(seed, *epoch, 1, thr) : ld_keep(seed, 0, 0, thr);
}

// n4 float4 groups; 16-bit copies (optional) as 4 x bf16 per group
// no __restrict__: out may alias keepv or skipv (in-place select of BatchNorm running statistics)
// outh (optional): the fp16 copy as well (the next post-LN layer's forward_f16 operand), from skiph /
// keeph or packed from the selected values
__global__ void __launch_bounds__(256) ld_select_k(const float4* skipv, const float4* keepv, float4* out,
                                                   const uint2* skip16, const uint2* keep16, uint2* out16,
                                                   int64_t n4, uint32_t thr, uint64_t seed,
                                                   const uint64_t* __restrict__ epoch, const uint2* skiph = nullptr,
                                                   const uint2* keeph = nullptr, uint2* outh = nullptr,
                                                   int inplace = 0) {
  const bool keep = dev_keep(seed, epoch, thr);
  if (keep && inplace) return;   // out (and its 16-bit copies) IS the kept tensor: nothing to move
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = keep ? keepv[i] : skipv[i];
    out[i] = v;
    if (out16) {
      const uint2* s16 = keep ? keep16 : skip16;
      out16[i] = s16 ? s16[i] : b2p_pack_bf16x4(v);
    }
    if (outh) {
      const uint2* sh = keep ? keeph : skiph;
      outh[i] = sh ? sh[i] : b2p_pack16x4(v, true);
    }
  }
}

__global__ void __launch_bounds__(256) ld_route_k(const float4* __restrict__ dout, float4* d_keep, float4* d_skip, int64_t n4, uint32_t thr,
                                                  uint64_t seed, const uint64_t* __restrict__ epoch) {
  const bool keep = dev_keep(seed, epoch, thr);
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  float4* to = keep ? d_keep : d_skip;     // the route is uniform: one full copy, one zero fill
  float4* zo = keep ? d_skip : d_keep;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    to[i] = dout[i];
    zo[i] = z;
  }
}

// the gate of one layer for this replay: flag = keep (1) or skip (0), the draw ld_select_k makes
__global__ void ld_flag_k(int32_t* flag, uint32_t thr, uint64_t seed, const uint64_t* __restrict__ epoch) {
  if (threadIdx.x == 0) *flag = dev_keep(seed, epoch, thr) ? 1 : 0;
}

inline unsigned grid_for(int64_t n4) {
  const int64_t b = (n4 + 255) / 256;
  return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace

extern "C" int b2p_layerdrop_keep(float p, uint64_t seed, uint64_t epoch, int has_epoch, int32_t* keep) {
  B2P_CHECK_ARG(keep != nullptr, "layerdrop_keep: NULL output");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "layerdrop_keep: p must be in [0,1)");
  *keep = ld_keep(seed, epoch, has_epoch, b2p_dropout_threshold(p)) ? 1 : 0;
  return 0;
}

extern "C" int b2p_layerdrop_select(const float* skip_val, const float* keep_val, float* out,
                                    const uint16_t* skip16, const uint16_t* keep16, uint16_t* out16, int64_t n,
                                    float p, uint64_t seed, b2p_stream_t stream) {
  return b2p_layerdrop_select_h(skip_val, keep_val, out, skip16, keep16, out16, nullptr, nullptr, nullptr, n, p, seed,
                                stream);
}

extern "C" int b2p_layerdrop_select_h(const float* skip_val, const float* keep_val, float* out,
                                      const uint16_t* skip16, const uint16_t* keep16, uint16_t* out16,
                                      const uint16_t* skiph, const uint16_t* keeph, uint16_t* outh, int64_t n,
                                      float p, uint64_t seed, b2p_stream_t stream) {
  B2P_CHECK_ARG((((uintptr_t)skiph | (uintptr_t)keeph | (uintptr_t)outh) & 7u) == 0,
                "layerdrop_select: fp16 buffers must be 8-byte aligned");
  B2P_CHECK_ARG(skip_val && keep_val && out, "layerdrop_select: NULL pointer");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "layerdrop_select: p must be in [0,1)");
  B2P_CHECK_ARG(n % 4 == 0, "layerdrop_select: n must be a multiple of 4");
  B2P_CHECK_ARG((((uintptr_t)skip_val | (uintptr_t)keep_val | (uintptr_t)out) & 15u) == 0,
                "layerdrop_select: fp32 buffers must be 16-byte aligned");
  B2P_CHECK_ARG((((uintptr_t)skip16 | (uintptr_t)keep16 | (uintptr_t)out16) & 7u) == 0,
                "layerdrop_select: bf16 buffers must be 8-byte aligned");
  const int64_t n4 = n / 4;
  if (n4 <= 0) return 0;
  hipLaunchKernelGGL(ld_select_k, dim3(grid_for(n4)), dim3(256), 0, (hipStream_t)stream, (const float4*)skip_val,
                     (const float4*)keep_val, (float4*)out, (const uint2*)skip16, (const uint2*)keep16, (uint2*)out16,
                     n4, b2p_dropout_threshold(p), seed, b2p_seed_epoch(), (const uint2*)skiph, (const uint2*)keeph,
                     (uint2*)outh, (int)(out == keep_val && out16 == keep16 && outh == keeph));
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layerdrop_route(const float* dout, float* d_keep, float* d_skip, int64_t n, float p, uint64_t seed,
                                   b2p_stream_t stream) {
  B2P_CHECK_ARG(dout && d_keep && d_skip, "layerdrop_route: NULL pointer");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "layerdrop_route: p must be in [0,1)");
  B2P_CHECK_ARG(n % 4 == 0, "layerdrop_route: n must be a multiple of 4");
  B2P_CHECK_ARG((((uintptr_t)dout | (uintptr_t)d_keep | (uintptr_t)d_skip) & 15u) == 0,
                "layerdrop_route: buffers must be 16-byte aligned");
  const int64_t n4 = n / 4;
  if (n4 <= 0) return 0;
  hipLaunchKernelGGL(ld_route_k, dim3(grid_for(n4)), dim3(256), 0, (hipStream_t)stream, (const float4*)dout,
                     (float4*)d_keep, (float4*)d_skip, n4, b2p_dropout_threshold(p), seed, b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layerdrop_flag(int32_t* flag, float p, uint64_t seed, b2p_stream_t stream) {
  B2P_CHECK_ARG(flag != nullptr, "layerdrop_flag: NULL flag");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "layerdrop_flag: p must be in [0,1)");
  hipLaunchKernelGGL(ld_flag_k, dim3(1), dim3(64), 0, (hipStream_t)stream, flag, b2p_dropout_threshold(p), seed,
                     b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}
