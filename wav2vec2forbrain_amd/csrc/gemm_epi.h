// GEMM epilogue shared by the fp32-operand kernel (gemm.hip) and the bf16 LDS-DMA kernel
// (gemm16.hip): alpha*acc + beta*C + bias(gather) -> pre_out -> act -> dropout -> act'(aux)
// -> residual -> C (fp32) and/or C16 (bf16 copy for the next GEMM's operand).
#pragma once
#include "common.h"
#include "../../include/b2p_hip.h"
#include <stdlib.h>

namespace {

// ------------------------------------------------------------------ epilogue
__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == B2P_ACT_GELU) return b2p_gelu(v);
  if (act == B2P_ACT_SOFTSIGN) return v / (1.0f + fabsf(v));
  if (act == B2P_ACT_SILU) return b2p_silu(v);
  return v;
}
__device__ __forceinline__ float act_grad(float x, int act) {
  if (act == B2P_ACT_GELU) return b2p_gelu_grad(x);
  if (act == B2P_ACT_SOFTSIGN) { const float d = 1.0f + fabsf(x); return 1.0f / (d * d); }
  if (act == B2P_ACT_SILU) return b2p_silu_grad(x);
  return 1.0f;
}

struct EpiArgs {
  b2p_epilogue e;
  int64_t M, N;
  uint32_t drop_thr;
  float drop_scale;
  int32_t vec4;   // every C-shaped tensor allows 16-B (C16: 8-B) accesses at n % 4 == 0
  const uint64_t* epoch;   // graph-replay dropout seed offset (b2p_seed_eff)
  const int32_t* gate;     // LayerDrop gate (b2p_gate): closed -> no K loop
  const int64_t* gates;    // per batch member z1: the member's gate pointer (b2p_gate_batch; 0 = open), or NULL
  uint32_t rk;             // gemm16 epilogue kind bits of this launch (EK_RUNTIME instantiations)
  uint32_t* tile_ctr;      // gemm16 split-K: per-tile arrival counters (zeroed per launch) -> the last
                           // K-slice workgroup of a tile sums the slabs itself (no reduce launch)
};

__device__ __forceinline__ void epilogue_store(const EpiArgs& a, int z, int z1, int z2, int m, int n,
                                               float acc) {
  if (m >= a.M || n >= a.N) return;
  const b2p_epilogue& e = a.e;
  const int64_t coff = (int64_t)z1 * e.cbs1 + (int64_t)z2 * e.cbs2 + (int64_t)m * e.ldc + n;
  float v = e.alpha * acc;
  if (e.beta != 0.0f) v += e.beta * e.C[coff];
  if (e.bias) v += e.bias[(e.bias_gather ? e.bias_gather[z1] : (int64_t)z1) * e.biasbs1 + n];
  if (e.pre_out) e.pre_out[coff] = v;
  if (e.pre16) e.pre16[coff] = b2p_bf16_bits(v);
  v = apply_act(v, e.act);
  if (e.drop_p > 0.0f) {
    const uint64_t idx = ((uint64_t)z * (uint64_t)a.M + (uint64_t)m) * (uint64_t)a.N + (uint64_t)n;
    v = b2p_keep(b2p_seed_eff(e.drop_seed, a.epoch), idx, a.drop_thr) ? v * a.drop_scale : 0.0f;
  }
  if (e.act_bwd != B2P_ACT_NONE) {
    const int64_t ao = (int64_t)z1 * e.abs1 + (int64_t)z2 * e.abs2 + (int64_t)m * e.ldaux + n;
    const float x = e.aux16 ? b2p_bf16_to_f32(e.aux16[ao]) : e.aux[ao];
    v *= act_grad(x, e.act_bwd);
  }
  if (e.residual) v += e.residual[(int64_t)z1 * e.rbs1 + (int64_t)z2 * e.rbs2 + (int64_t)m * e.ldr + n];
  if (e.C) e.C[coff] = v;
  if (e.C16) e.C16[coff] = b2p_16_bits(v, e.flags & B2P_EPI_C16_FP16);
  if (e.C16b) e.C16b[coff] = b2p_bf16_bits(v);
}

// Four consecutive columns n .. n+3 of row m (n % 4 == 0), vectorised when ea.vec4 is set.
// Returns the final values (0 outside the matrix) for the fused column sums.
__device__ __forceinline__ float4 epilogue_store4(const EpiArgs& a, int z, int z1, int z2, int m, int n, float4 acc) {
  if (m >= a.M || n >= a.N) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (!a.vec4 || n + 4 > a.N) {
    epilogue_store(a, z, z1, z2, m, n, acc.x);
    if (n + 1 < a.N) epilogue_store(a, z, z1, z2, m, n + 1, acc.y);
    if (n + 2 < a.N) epilogue_store(a, z, z1, z2, m, n + 2, acc.z);
    if (n + 3 < a.N) epilogue_store(a, z, z1, z2, m, n + 3, acc.w);
    return make_float4(0.f, 0.f, 0.f, 0.f);   // (colsum_part requires vec4, checked on the host)
  }
  const b2p_epilogue& e = a.e;
  const int64_t coff = (int64_t)z1 * e.cbs1 + (int64_t)z2 * e.cbs2 + (int64_t)m * e.ldc + n;
  float v[4] = {e.alpha * acc.x, e.alpha * acc.y, e.alpha * acc.z, e.alpha * acc.w};
  if (e.beta != 0.0f) {
    const float4 c = *reinterpret_cast<const float4*>(e.C + coff);
    v[0] += e.beta * c.x; v[1] += e.beta * c.y; v[2] += e.beta * c.z; v[3] += e.beta * c.w;
  }
  if (e.bias) {
    const float4 b = *reinterpret_cast<const float4*>(
        e.bias + (e.bias_gather ? e.bias_gather[z1] : (int64_t)z1) * e.biasbs1 + n);
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
  }
  if (e.pre_out) *reinterpret_cast<float4*>(e.pre_out + coff) = make_float4(v[0], v[1], v[2], v[3]);
  if (e.pre16) *reinterpret_cast<uint2*>(e.pre16 + coff) = b2p_pack_bf16x4(make_float4(v[0], v[1], v[2], v[3]));
  if (e.act == B2P_ACT_GELU) {   // packed: two elements per VALU instruction
    const b2p_f2 g0 = b2p_gelu2(b2p_f2{v[0], v[1]}), g1 = b2p_gelu2(b2p_f2{v[2], v[3]});
    v[0] = g0.x; v[1] = g0.y; v[2] = g1.x; v[3] = g1.y;
  } else if (e.act != B2P_ACT_NONE) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = apply_act(v[q], e.act);
  }
  if (e.drop_p > 0.0f) {
    const uint64_t idx = ((uint64_t)z * (uint64_t)a.M + (uint64_t)m) * (uint64_t)a.N + (uint64_t)n;
    const uint64_t sd = b2p_seed_eff(e.drop_seed, a.epoch);
    bool k[4];
    b2p_keep4(sd, idx, a.drop_thr, k);   // idx % 4 == 0 (vec4: N % 4 == 0, n % 4 == 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = k[q] ? v[q] * a.drop_scale : 0.0f;
  }
  if (e.act_bwd != B2P_ACT_NONE) {
    const int64_t ao = (int64_t)z1 * e.abs1 + (int64_t)z2 * e.abs2 + (int64_t)m * e.ldaux + n;
    float4 x;
    if (e.aux16) {
      const uint2 h = *reinterpret_cast<const uint2*>(e.aux16 + ao);
      x = make_float4(b2p_bf16_to_f32((uint16_t)(h.x & 0xffffu)), b2p_bf16_to_f32((uint16_t)(h.x >> 16)),
                      b2p_bf16_to_f32((uint16_t)(h.y & 0xffffu)), b2p_bf16_to_f32((uint16_t)(h.y >> 16)));
    } else {
      x = *reinterpret_cast<const float4*>(e.aux + ao);
    }
    if (e.act_bwd == B2P_ACT_GELU) {
      const b2p_f2 g0 = b2p_gelu_grad2(b2p_f2{x.x, x.y}), g1 = b2p_gelu_grad2(b2p_f2{x.z, x.w});
      v[0] *= g0.x; v[1] *= g0.y; v[2] *= g1.x; v[3] *= g1.y;
    } else {
      v[0] *= act_grad(x.x, e.act_bwd); v[1] *= act_grad(x.y, e.act_bwd);
      v[2] *= act_grad(x.z, e.act_bwd); v[3] *= act_grad(x.w, e.act_bwd);
    }
  }
  if (e.residual) {
    const float4 r = *reinterpret_cast<const float4*>(
        e.residual + (int64_t)z1 * e.rbs1 + (int64_t)z2 * e.rbs2 + (int64_t)m * e.ldr + n);
    v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
  }
  if (e.C) *reinterpret_cast<float4*>(e.C + coff) = make_float4(v[0], v[1], v[2], v[3]);
  if (e.C16) *reinterpret_cast<uint2*>(e.C16 + coff) = b2p_pack16x4(make_float4(v[0], v[1], v[2], v[3]),
                                                                       e.flags & B2P_EPI_C16_FP16);
  if (e.C16b) *reinterpret_cast<uint2*>(e.C16b + coff) = b2p_pack_bf16x4(make_float4(v[0], v[1], v[2], v[3]));
  return make_float4(v[0], v[1], v[2], v[3]);
}

// C[z](m,n) = alpha * sum_s slab[z][s](m,n) + beta * C_old ; deterministic slice order
__global__ void splitk_reduce(const float* __restrict__ ws, int ks, int64_t M, int64_t N, int nz2,
                              b2p_epilogue e, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t MN = M * N;
  const int64_t z = i / MN, r = i - z * MN;
  const int64_t m = r / N, n = r - m * N;
  const float* p = ws + z * ks * MN + r;
  float s = 0.f;
  for (int q = 0; q < ks; ++q) s += p[(int64_t)q * MN];
  const int64_t z1 = z / nz2, z2 = z - z1 * nz2;
  const int64_t coff = z1 * e.cbs1 + z2 * e.cbs2 + m * e.ldc + n;
  float v = e.alpha * s;
  if (e.beta != 0.f) v += e.beta * e.C[coff];
  if (e.C) e.C[coff] = v;
  if (e.C16) e.C16[coff] = b2p_16_bits(v, e.flags & B2P_EPI_C16_FP16);
}

// the same with 4 consecutive columns per thread (N % 4 == 0, ldc % 4 == 0, cbs % 4 == 0, C 16-B and
// C16 8-B aligned): 16-B slab loads, 4x fewer instructions per byte
__global__ void __launch_bounds__(256) splitk_reduce4(const float* __restrict__ ws, int ks, int64_t M, int64_t N,
                                                      int nz2, b2p_epilogue e, int64_t total4) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 >= total4) return;
  const int64_t MN = M * N, i = 4 * i4;
  const int64_t z = i / MN, r = i - z * MN;
  const int64_t m = r / N, n = r - m * N;
  const float* p = ws + z * ks * MN + r;
  float4 s = *reinterpret_cast<const float4*>(p);
  for (int q = 1; q < ks; ++q) {
    const float4 v = *reinterpret_cast<const float4*>(p + (int64_t)q * MN);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const int64_t z1 = z / nz2, z2 = z - z1 * nz2;
  const int64_t coff = z1 * e.cbs1 + z2 * e.cbs2 + m * e.ldc + n;
  float4 v = make_float4(e.alpha * s.x, e.alpha * s.y, e.alpha * s.z, e.alpha * s.w);
  if (e.beta != 0.f) {
    const float4 c = *reinterpret_cast<const float4*>(e.C + coff);
    v.x += e.beta * c.x; v.y += e.beta * c.y; v.z += e.beta * c.z; v.w += e.beta * c.w;
  }
  if (e.C) *reinterpret_cast<float4*>(e.C + coff) = v;
  if (e.C16) *reinterpret_cast<uint2*>(e.C16 + coff) = b2p_pack16x4(v, e.flags & B2P_EPI_C16_FP16);
}

inline EpiArgs make_epi_args(const b2p_gemm_desc& d) {
  EpiArgs ea;
  ea.e = d.ep;
  ea.M = d.M;
  ea.N = d.N;
  ea.drop_thr = b2p_dropout_threshold(d.ep.drop_p);
  ea.drop_scale = d.ep.drop_p > 0.f ? 1.0f / (1.0f - d.ep.drop_p) : 1.0f;
  const b2p_epilogue& e = d.ep;
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  auto s4 = [](int64_t x) { return x % 4 == 0; };
  bool v = d.N % 4 == 0 && s4(e.ldc) && s4(e.cbs1) && s4(e.cbs2) && a16(e.C) && a16(e.pre_out) &&
           ((uintptr_t)e.C16 & 7u) == 0;
  if (e.bias) v = v && a16(e.bias) && s4(e.biasbs1);
  if (e.act_bwd != B2P_ACT_NONE)
    v = v && (e.aux16 ? ((uintptr_t)e.aux16 & 7u) == 0 : a16(e.aux)) && s4(e.ldaux) && s4(e.abs1) && s4(e.abs2);
  if (e.pre16) v = v && ((uintptr_t)e.pre16 & 7u) == 0;
  if (e.C16b) v = v && ((uintptr_t)e.C16b & 7u) == 0;
  if (e.residual) v = v && a16(e.residual) && s4(e.ldr) && s4(e.rbs1) && s4(e.rbs2);
  ea.vec4 = v ? 1 : 0;
  ea.epoch = b2p_seed_epoch();
  ea.gate = b2p_gate();
  ea.gates = b2p_gate_batch();
  ea.rk = 0;
  ea.tile_ctr = nullptr;
  return ea;
}

}  // namespace

// bf16-operand (LDS-DMA) GEMM launcher, gemm16.hip; arguments already validated by b2p_gemm.
int b2p_gemm16_launch(const b2p_gemm_desc& d, hipStream_t st);
// true when the gemm16 launch of d sums its split-K slabs itself (no reduce launch after it)
bool gemm16_splitk_fused(const b2p_gemm_desc& d);
