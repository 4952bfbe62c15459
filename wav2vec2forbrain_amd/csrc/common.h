// Shared device/host helpers for the b2p2t HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// fp32 -> bf16 bits, round-to-nearest-even (plain cast: v_cvt_pk_bf16_f32, keeps NaN a NaN)
__device__ __forceinline__ uint16_t b2p_bf16_bits(float v) {
  return __builtin_bit_cast(uint16_t, (__bf16)v);
}
__device__ __forceinline__ uint2 b2p_pack_bf16x4(float4 v) {
  return make_uint2((uint32_t)b2p_bf16_bits(v.x) | ((uint32_t)b2p_bf16_bits(v.y) << 16),
                    (uint32_t)b2p_bf16_bits(v.z) | ((uint32_t)b2p_bf16_bits(v.w) << 16));
}
// fp16 with saturation: finite values beyond fp16's range clamp to +-65504 instead of becoming
// infinities in a GEMM operand (the Conformer's fp16 forward operands, Fn.forward_f16); NaN stays NaN
__device__ __forceinline__ float b2p_f16_sat(float v) { return fabsf(v) > 65504.f ? copysignf(65504.f, v) : v; }
__device__ __forceinline__ uint16_t b2p_f16_bits(float v) { return __builtin_bit_cast(uint16_t, (_Float16)b2p_f16_sat(v)); }
// 16-bit bits of v: fp16 when half, else bf16
__device__ __forceinline__ uint16_t b2p_16_bits(float v, bool half) { return half ? b2p_f16_bits(v) : b2p_bf16_bits(v); }
__device__ __forceinline__ uint2 b2p_pack16x4(float4 v, bool half) {
  return make_uint2((uint32_t)b2p_16_bits(v.x, half) | ((uint32_t)b2p_16_bits(v.y, half) << 16),
                    (uint32_t)b2p_16_bits(v.z, half) | ((uint32_t)b2p_16_bits(v.w, half) << 16));
}
// 8 fp16 values in a 16-bit container vector (the data movement is the same as bf16's) and the fp16
// MFMA on such containers: the GRU forward recurrences (gru16 / grumc) keep W_hh and h in fp16 —
// both are bounded (|h| < 1, W_hh ~ U(-1/sqrt(H), 1/sqrt(H))) and get 3 more significant bits
typedef _Float16 b2p_f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x8 b2p_pack8_f16(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  const b2p_f16x8 r = {(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
                       (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
  return __builtin_bit_cast(bf16x8, r);
}
__device__ __forceinline__ f32x4 b2p_mfma_f16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(b2p_f16x8, a), __builtin_bit_cast(b2p_f16x8, b), c,
                                                0, 0, 0);
}
__device__ __forceinline__ uint2 b2p_pack_f16x4(float4 v) {
  return make_uint2((uint32_t)b2p_f16_bits(v.x) | ((uint32_t)b2p_f16_bits(v.y) << 16),
                    (uint32_t)b2p_f16_bits(v.z) | ((uint32_t)b2p_f16_bits(v.w) << 16));
}
__device__ __forceinline__ float b2p_bf16_to_f32(uint16_t b) {
  return __builtin_bit_cast(float, (uint32_t)b << 16);
}

// ---------------------------------------------------------------------------
// error reporting: every C-ABI entry returns 0 on success, nonzero on failure
// and leaves a message retrievable through b2p_last_error().
// ---------------------------------------------------------------------------
// device counter added to every dropout seed (NULL: none); set by b2p_set_seed_epoch (lib.cpp)
const uint64_t* b2p_seed_epoch();
// LayerDrop gate set by b2p_set_gate (lib.cpp): GEMMs under a closed gate skip their K loop (acc = 0,
// epilogue still runs, so every output stays finite), fused attention skips its work
const int32_t* b2p_gate();
// per-member gates of a batched launch (b2p_set_gate_batch): device int64[nz1] of int32* (0 = open)
const int64_t* b2p_gate_batch();
__device__ __forceinline__ bool b2p_gated_off(const int32_t* gate) { return gate && *gate == 0; }
void b2p_set_error(const char* fmt, ...);

#define B2P_CHECK_ARG(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      b2p_set_error(__VA_ARGS__);                \
      return 1;                                  \
    }                                            \
  } while (0)

#define B2P_CHECK_HIP(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      b2p_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                    __FILE__, __LINE__);                                      \
      return 2;                                                               \
    }                                                                         \
  } while (0)

#define B2P_CHECK_LAUNCH() B2P_CHECK_HIP(hipGetLastError())

// ---------------------------------------------------------------------------
// device math
// ---------------------------------------------------------------------------
// erf(z) for z >= 0 given e = exp(-z*z): Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7), one
// reciprocal + four FMAs, branch-free (the library erff is a ~30-instruction piecewise polynomial;
// in the GEMM epilogues the GELU / GELU' of every FFN element is VALU work beside the MFMAs).
// Every step is an explicit FMA / multiply so the packed two-element forms below (v_pk_fma_f32 /
// v_pk_mul_f32: half the VALU issue of the epilogue's GELU) are bit-identical to the scalar ones.
__device__ __forceinline__ float b2p_erf_pos(float z, float e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  return fmaf(-(p * t), e, 1.0f);
}
// Phi(x) = 0.5 * (1 + erf(x / sqrt 2)), with exp(-x^2/2) returned for the GELU derivative
__device__ __forceinline__ float b2p_phi(float x, float& e) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  e = __expf(-(z * z));
  const float er = b2p_erf_pos(z, e);
  return fmaf(0.5f, copysignf(er, x), 0.5f);
}
__device__ __forceinline__ float b2p_gelu(float x) {
  // exact-erf GELU (transformers ACT2FN["gelu"] == torch.nn.functional.gelu), erf to 1.5e-7
  float e;
  return x * b2p_phi(x, e);
}
__device__ __forceinline__ float b2p_gelu_grad(float x) {
  float e;
  const float cdf = b2p_phi(x, e);
  return fmaf(x * 0.39894228040143267794f, e, cdf);   // Phi(x) + x * pdf(x), pdf = e / sqrt(2 pi)
}
typedef float b2p_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ b2p_f2 b2p_fma2(b2p_f2 a, b2p_f2 b, b2p_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ b2p_f2 b2p_splat2(float v) { return b2p_f2{v, v}; }
// Phi of two elements (packed): same operation sequence as b2p_phi
__device__ __forceinline__ b2p_f2 b2p_phi2(b2p_f2 x, b2p_f2& e) {
  const b2p_f2 z = b2p_f2{fabsf(x.x), fabsf(x.y)} * b2p_splat2(0.70710678118654752440f);
  const b2p_f2 nz = -(z * z);
  e = b2p_f2{__expf(nz.x), __expf(nz.y)};
  const b2p_f2 d = b2p_fma2(b2p_splat2(0.3275911f), z, b2p_splat2(1.0f));
  const b2p_f2 t = b2p_f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  b2p_f2 p = b2p_fma2(b2p_splat2(1.061405429f), t, b2p_splat2(-1.453152027f));
  p = b2p_fma2(p, t, b2p_splat2(1.421413741f));
  p = b2p_fma2(p, t, b2p_splat2(-0.284496736f));
  p = b2p_fma2(p, t, b2p_splat2(0.254829592f));
  const b2p_f2 er = b2p_fma2(-(p * t), e, b2p_splat2(1.0f));
  return b2p_fma2(b2p_splat2(0.5f), b2p_f2{copysignf(er.x, x.x), copysignf(er.y, x.y)}, b2p_splat2(0.5f));
}
__device__ __forceinline__ b2p_f2 b2p_gelu2(b2p_f2 x) {
  b2p_f2 e;
  return x * b2p_phi2(x, e);
}
__device__ __forceinline__ b2p_f2 b2p_gelu_grad2(b2p_f2 x) {
  b2p_f2 e;
  const b2p_f2 cdf = b2p_phi2(x, e);
  return b2p_fma2(x * b2p_splat2(0.39894228040143267794f), e, cdf);
}
__device__ __forceinline__ float b2p_sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float b2p_silu(float x) { return x * b2p_sigmoid(x); }
__device__ __forceinline__ float b2p_silu_grad(float x) {
  const float s = b2p_sigmoid(x);
  return s * (1.0f + x * (1.0f - s));
}

// Counter-based dropout mask (stateless, so backward regenerates the forward mask from
// (seed, element index) instead of storing it). lowbias32 (a 32-bit bijection with two
// multiplies) applied twice over the index, keyed by the seed: ~4 v_mul per element instead of
// splitmix64's 64-bit multiplies (the attention kernels draw ~24M masks per layer and pass).
__device__ __forceinline__ uint32_t b2p_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t b2p_hash(uint64_t seed, uint64_t idx) {
  const uint32_t k = (uint32_t)seed ^ b2p_mix32((uint32_t)(seed >> 32) + 0x9E3779B9u);   // per-launch key
#ifdef B2P_HASH_1R   // measurement variant: one mixing round (tools/build_variant.sh)
  return b2p_mix32((uint32_t)idx ^ k ^ ((uint32_t)(idx >> 32) * 0x85EBCA6Bu));
#else
  return b2p_mix32(b2p_mix32((uint32_t)idx ^ k) + (uint32_t)(idx >> 32) * 0x85EBCA6Bu + k);
#endif
}
// keep-probability threshold: keep iff hash >= thr, thr = round(p * 2^32)
// Graph-replayed steps: the host-drawn seed of every dropout call is offset by a device-resident
// step counter (b2p_set_seed_epoch), so a captured step draws new masks on every replay. NULL (the
// eager default) leaves the seed unchanged.
__device__ __forceinline__ uint64_t b2p_seed_eff(uint64_t seed, const uint64_t* epoch) {
  return epoch ? seed + 0x9E3779B97F4A7C15ull * (*epoch) : seed;
}
// One hash serves two consecutive elements: element idx keeps iff its 16-bit half of
// b2p_hash(seed, idx >> 1) (low half for even idx) is >= thr16 = round(p * 2^16), so the keep
// probability is exact to 2^-16 and a 4-element group costs two hashes (b2p_keep4).
__device__ __forceinline__ uint32_t b2p_thr16(uint32_t thr) { return (thr >> 16) + ((thr >> 15) & 1u); }
__device__ __forceinline__ bool b2p_keep(uint64_t seed, uint64_t idx, uint32_t thr) {
  const uint32_t h = b2p_hash(seed, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= b2p_thr16(thr);
}
// keep bits of elements idx .. idx+3, idx even
__device__ __forceinline__ void b2p_keep4(uint64_t seed, uint64_t idx, uint32_t thr, bool k[4]) {
  const uint32_t t = b2p_thr16(thr);
  const uint32_t h0 = b2p_hash(seed, idx >> 1), h1 = b2p_hash(seed, (idx >> 1) + 1);
  k[0] = (h0 & 0xFFFFu) >= t;
  k[1] = (h0 >> 16) >= t;
  k[2] = (h1 & 0xFFFFu) >= t;
  k[3] = (h1 >> 16) >= t;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline uint32_t b2p_dropout_threshold(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) return 0xFFFFFFFFu;
  return (uint32_t)t;
}
