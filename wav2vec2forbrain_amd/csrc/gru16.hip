// Persistent bf16-MFMA GRU recurrence (nn.GRU semantics, gate order r, z, n) for the brain-feature
// encoder (reference src/model/brain_feature_extractor.py:39-47, 56-68), bf16 precision mode.
//
// One workgroup runs the WHOLE time loop of one direction for 16 batch rows: W_hh never leaves the
// CU (r/z gate rows as MFMA A-fragments in VGPRs, n gate rows in LDS), h_{t-1} is exchanged
// between the CU's waves through a double-buffered LDS image, so a time step costs one
// workgroup barrier instead of a kernel launch and a W_hh re-read from L2. Per step and CU:
//   gates^T (3H x 16) = W_hh (3H x H) . h_{t-1}^T (H x 16)   -- v_mfma_f32_16x16x32_f16, fp32 acc
// The forward's operands are fp16 (W_hh and h are bounded, so fp16's 11 significant bits cost no
// range; bf16 operands here put 3.7e-4 of relative CTC-loss error into the Conformer-large step,
// tools/traj_err.py); the backward's are bf16 (gradients span magnitudes below fp16's range).
// Wave w owns hidden units [32w, 32w+32) (two 16-unit blocks) for all three gates, so the gate
// nonlinearities run on the accumulators in registers (lane: batch = lane&15, 4 units per block).
// h, the gate activations and everything stored stay fp32; only the MFMA operands are 16-bit.
// Backward (BPTT) is the mirror image: dh_rec (H x 16) = W_hh^T (H x 3H) . dgh_{s+1}^T (3H x 16).
//
// Per-step tensors use a LANE-NATIVE layout ("LN"): for direction d, batch group bg (16 rows),
// processing step s, unit block ub (16 units) and record r (a gate), the 64 lanes' float4s are
// contiguous, so every per-step load/store is one coalesced 1 KB wave access (the standard
// (B, T, ndir*R*H) layout costs 16 half-lines per access and measured 2x the step time).
//   LN float offset = (((((d*NBG + bg)*T + s)*U + ub)*R + r)*64 + lane)*4 + i,
//   lane = (b % 16) + 16*((j % 16) / 4), i = j % 4, ub = j / 16, U = H/16, s = t (d=0) or T-1-t.
// b2p_gru_lane_permute converts between the two layouts (bulk, HBM-bound).
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {
constexpr int BG = 16;   // batch rows per workgroup = MFMA N

__device__ __forceinline__ bf16x8 pack8_strided(const float* p, int64_t stride) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)p[j * stride];
  return r;
}
__device__ __forceinline__ void store_bf16x4(uint16_t* dst, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(dst) = b2p_pack_bf16x4(make_float4(a, b, c, d));
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float comp(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ f32x4 to_acc(const float4& v) { return f32x4{v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ float4 mul4(const float4& a, const float4& b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}

// Raw buffer access (32-bit byte offsets, hardware range check): loads/stores stay unconditional
// (exact vmcnt counting) and an out-of-range load returns 0 (null h0).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mkbuf(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, p ? bytes : 0u, 0x00020000);
}
__device__ __forceinline__ float4 bld4(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void bst4(rsrc_t r, uint32_t off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, off,
                                         0, 0);
}

// fast gate nonlinearities (v_exp_f32 + v_rcp_f32; ~1e-6 relative, well inside the bf16-mode budget)
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)); }
// workgroup barrier for the LDS hand-off only: waits for this wave's LDS traffic (lgkmcnt) but not
// for its outstanding global stores (__syncthreads would drain vmcnt every time step)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int H>
constexpr size_t fwd_lds_bytes() {
  return (size_t)(H / 32) * 2 * (H / 32) * 64 * 16 + 2 * BG * (H + 8) * 2 + H * 4;
}
template <int H>
constexpr size_t bwd_lds_bytes() {
  return (size_t)(H / 32) * 2 * (H / 32) * 64 * 16 + BG * (3 * H + 8) * 2;
}
// byte offset of (d, bg, s) record block in an LN tensor with R records; per-lane part added by caller
__device__ __forceinline__ uint32_t ln_step(int d, int bg, int nbg, int T, int s, int H, int R) {
  return (uint32_t)((((int64_t)d * nbg + bg) * T + s) * (H / 16) * R * 1024);
}

// ------------------------------------------------------------------------------------------ forward
// giL: LN(R=3) of x W_ih^T + b_ih + (b_hr, b_hz, 0) (b_hh's r/z parts folded by the caller: they
// only ever appear summed with it); bhh [ndir][3H] (null = 0) is read for b_hn only; h0 [ndir][B][H]
// or null. Outputs hL: LN(R=1) of h; savL: LN(R=4) of (r, z, n, W_hn h + b_hn).
// DIAG (tools/gru_probe.hip ablations only; 0 in the library): 1 no MFMAs, 2 no gate nonlinearities,
// 4 no global stores, 8 no workgroup barrier, 16 no gi loads. SPLIT: the two unit blocks' K loops one
// after the other, block 0's gate math and stores interleaved with block 1's MFMAs
template <int H, int DIAG = 0, bool SPLIT = false>
__global__ void __launch_bounds__(H * 2) gru16_fwd(const float* __restrict__ giL, const float* __restrict__ whh,
                                                   const float* __restrict__ bhh, const float* __restrict__ h0,
                                                   float* __restrict__ hL, float* __restrict__ savL, int B, int T,
                                                   int ndir) {
  constexpr int KS = H / 32;     // k-steps
  constexpr int NW = H / 32;     // waves
  constexpr int HP = H + 8;      // bf16 row pitch of the h image (16-B stagger per row)
  constexpr int G3 = 3 * H;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16x8* wn_lds = reinterpret_cast<bf16x8*>(smem);                              // [NW][2][KS][64]
  uint16_t* hb = reinterpret_cast<uint16_t*>(smem + (size_t)NW * 2 * KS * 64 * 16);   // [2][BG][HP]
  float* bias = reinterpret_cast<float*>(hb + 2 * BG * HP);                      // [H] b_hn

  const int d = blockIdx.y, bg = blockIdx.x, nbg = gridDim.x;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lr = l & 15, lq = l >> 4;
  const float* W = whh + (int64_t)d * G3 * H;
  const int b = bg * BG + lr;
  const bool bok = b < B;

  bf16x8 wr[2][KS], wz[2][KS];
#pragma unroll
  for (int ub = 0; ub < 2; ++ub) {
    const int row = (2 * w + ub) * 16 + lr;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float* p = W + (int64_t)row * H + 32 * s + 8 * lq;
      wr[ub][s] = b2p_pack8_f16(p);
      wz[ub][s] = b2p_pack8_f16(p + (int64_t)H * H);
      wn_lds[((w * 2 + ub) * KS + s) * 64 + l] = b2p_pack8_f16(p + 2 * (int64_t)H * H);
    }
  }
  for (int i = tid; i < H; i += H * 2) bias[i] = bhh ? bhh[(int64_t)d * G3 + 2 * H + i] : 0.f;
  float hp[2][4];
#pragma unroll
  for (int ub = 0; ub < 2; ++ub) {
    const int j0 = (2 * w + ub) * 16 + 4 * lq;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bok && h0) v = ld4(h0 + ((int64_t)d * B + b) * H + j0);
    hp[ub][0] = v.x; hp[ub][1] = v.y; hp[ub][2] = v.z; hp[ub][3] = v.w;
    *reinterpret_cast<uint2*>(hb + lr * HP + j0) = b2p_pack_f16x4(v);
  }
  __syncthreads();

  const uint32_t nbytes1 = (uint32_t)((int64_t)ndir * nbg * T * H * 16 * 4);   // LN bytes per record
  const rsrc_t gi_r = mkbuf(giL, 3 * nbytes1);
  const rsrc_t h_r = mkbuf(hL, nbytes1);
  const rsrc_t sv_r = mkbuf(savL, 4 * nbytes1);
  // LN byte offset of this lane inside a step block with R records: R * wb + (ub * R + r) KB + lo
  const uint32_t wb = (uint32_t)(2 * w) * 1024u, lo = (uint32_t)l * 16u, lane_b = wb + lo;
  // gi is prefetched one time step ahead: its r/z parts become the MFMA accumulator inputs (they
  // are summed with W_h{r,z} h anyway), its n part waits for r
  auto load_gi = [&](int s, float4 (&g)[2][3]) {
    if (DIAG & 16) {
#pragma unroll
      for (int ub = 0; ub < 2; ++ub)
#pragma unroll
        for (int q = 0; q < 3; ++q) g[ub][q] = make_float4(0.01f * s, 0.f, 0.f, 0.f);
      return;
    }
    const uint32_t o = ln_step(d, bg, nbg, T, s, H, 3) + 3 * wb + lo;
#pragma unroll
    for (int ub = 0; ub < 2; ++ub)
#pragma unroll
      for (int q = 0; q < 3; ++q) g[ub][q] = bld4(gi_r, o + (uint32_t)(ub * 3 + q) * 1024u);
  };
  // one time step; gc = gi of this step (prefetched), gx receives gi of the next step. The loop is
  // unrolled by two with the buffers swapped, so no register copy of a pending load (which would
  // force an early vmcnt drain) is needed.
  auto step = [&](int s, float4 (&gc)[2][3], float4 (&gx)[2][3]) {
    f32x4 acc[2][3];
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) {
      acc[ub][0] = to_acc(gc[ub][0]);
      acc[ub][1] = to_acc(gc[ub][1]);
      acc[ub][2] = *reinterpret_cast<const f32x4*>(bias + (2 * w + ub) * 16 + 4 * lq);
    }
    load_gi(s + 1 < T ? s + 1 : s, gx);   // last step re-reads itself (unused): load stays unconditional
    const uint16_t* hcur = hb + (s & 1) * BG * HP + lr * HP + 8 * lq;
    const bf16x8* wnl = wn_lds + (w * 2) * KS * 64 + l;
    // LDS fragments one k-step ahead of the MFMAs; the sched barrier keeps the compiler from
    // hoisting every k-step's loads (that spills the VGPR-resident W_hh fragments)
    uint16_t* hnxt = hb + ((s + 1) & 1) * BG * HP;
    const uint32_t oh = ln_step(d, bg, nbg, T, s, H, 1) + lane_b;
    const uint32_t osv = ln_step(d, bg, nbg, T, s, H, 4) + 4 * wb + lo;
    // gate math, stores and h hand-off of unit block ub; part = -1: all of it, else the slice of it that
    // rides along k-step `part` of the other block's MFMAs (elements 0-3, then the stores)
    float rr[2][4], zz[2][4], nn[2][4], hh[2][4];
    auto finish = [&](int ub, int part) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (part >= 0 && part != i) continue;
        if (DIAG & 2) {
          rr[ub][i] = acc[ub][0][i];
          zz[ub][i] = acc[ub][1][i];
          nn[ub][i] = comp(gc[ub][2], i) + rr[ub][i] * acc[ub][2][i];
        } else {
          rr[ub][i] = sigm(acc[ub][0][i]);
          zz[ub][i] = sigm(acc[ub][1][i]);
          nn[ub][i] = tanh_fast(comp(gc[ub][2], i) + rr[ub][i] * acc[ub][2][i]);
        }
        hh[ub][i] = bok ? (1.f - zz[ub][i]) * nn[ub][i] + zz[ub][i] * hp[ub][i] : 0.f;
        hp[ub][i] = hh[ub][i];
      }
      const int j0 = (2 * w + ub) * 16 + 4 * lq;
      const uint32_t o = osv + (uint32_t)ub * 4096u;
      if (part < 0 || part == 4) {
        *reinterpret_cast<uint2*>(hnxt + lr * HP + j0) =
            b2p_pack_f16x4(make_float4(hh[ub][0], hh[ub][1], hh[ub][2], hh[ub][3]));
        if (!(DIAG & 4) || s == T - 1)
          bst4(h_r, oh + (uint32_t)ub * 1024u, make_float4(hh[ub][0], hh[ub][1], hh[ub][2], hh[ub][3]));
      }
      if ((part < 0 || part == 5) && (!(DIAG & 4) || s == T - 1)) {
        bst4(sv_r, o, make_float4(rr[ub][0], rr[ub][1], rr[ub][2], rr[ub][3]));
        bst4(sv_r, o + 1024u, make_float4(zz[ub][0], zz[ub][1], zz[ub][2], zz[ub][3]));
      }
      if ((part < 0 || part == 6) && (!(DIAG & 4) || s == T - 1)) {
        bst4(sv_r, o + 2048u, make_float4(nn[ub][0], nn[ub][1], nn[ub][2], nn[ub][3]));
        bst4(sv_r, o + 3072u, make_float4(acc[ub][2][0], acc[ub][2][1], acc[ub][2][2], acc[ub][2][3]));
      }
    };
    bf16x8 bf = *reinterpret_cast<const bf16x8*>(hcur);
    bf16x8 an0 = wnl[0], an1 = wnl[KS * 64];
    if (SPLIT && !(DIAG & 1)) {
      // block 0's K loop, then block 1's with block 0's gate math / stores interleaved one slice per
      // k-step: the VALU work of one block runs while the other block's MFMAs occupy the matrix core
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 bfn = bf, an0n = an0;
        if (ks + 1 < KS) {
          bfn = *reinterpret_cast<const bf16x8*>(hcur + 32 * (ks + 1));
          an0n = wnl[(ks + 1) * 64];
        }
        acc[0][0] = b2p_mfma_f16(wr[0][ks], bf, acc[0][0]);
        acc[0][1] = b2p_mfma_f16(wz[0][ks], bf, acc[0][1]);
        acc[0][2] = b2p_mfma_f16(an0, bf, acc[0][2]);
        __builtin_amdgcn_sched_barrier(0);
        bf = bfn; an0 = an0n;
      }
      bf = *reinterpret_cast<const bf16x8*>(hcur);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 bfn = bf, an1n = an1;
        if (ks + 1 < KS) {
          bfn = *reinterpret_cast<const bf16x8*>(hcur + 32 * (ks + 1));
          an1n = wnl[(KS + ks + 1) * 64];
        }
        acc[1][0] = b2p_mfma_f16(wr[1][ks], bf, acc[1][0]);
        acc[1][1] = b2p_mfma_f16(wz[1][ks], bf, acc[1][1]);
        acc[1][2] = b2p_mfma_f16(an1, bf, acc[1][2]);
        if (KS >= 8) finish(0, ks);   // parts 0-6
        __builtin_amdgcn_sched_barrier(0);
        bf = bfn; an1 = an1n;
      }
      if (KS < 8) finish(0, -1);
      finish(1, -1);
    }
#pragma unroll
    for (int ks = 0; ks < ((DIAG & 1) || SPLIT ? 0 : KS); ++ks) {
      bf16x8 bfn = bf, an0n = an0, an1n = an1;
      if (ks + 1 < KS) {
        bfn = *reinterpret_cast<const bf16x8*>(hcur + 32 * (ks + 1));
        an0n = wnl[(ks + 1) * 64];
        an1n = wnl[(KS + ks + 1) * 64];
      }
      acc[0][0] = b2p_mfma_f16(wr[0][ks], bf, acc[0][0]);
      acc[0][1] = b2p_mfma_f16(wz[0][ks], bf, acc[0][1]);
      acc[0][2] = b2p_mfma_f16(an0, bf, acc[0][2]);
      acc[1][0] = b2p_mfma_f16(wr[1][ks], bf, acc[1][0]);
      acc[1][1] = b2p_mfma_f16(wz[1][ks], bf, acc[1][1]);
      acc[1][2] = b2p_mfma_f16(an1, bf, acc[1][2]);
      __builtin_amdgcn_sched_barrier(0);
      bf = bfn; an0 = an0n; an1 = an1n;
    }
    if (!SPLIT || (DIAG & 1)) {
      finish(0, -1);
      finish(1, -1);
    }
    if (DIAG & 8)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else
      lds_barrier();
  };
  float4 ga[2][3], gb2[2][3];
  load_gi(0, ga);
  int s = 0;
  for (; s + 1 < T; s += 2) {
    step(s, ga, gb2);
    step(s + 1, gb2, ga);
  }
  if (s < T) step(s, ga, gb2);
}

// ----------------------------------------------------------------------------------------- backward
// Processing step s (direction d's own time order) runs backwards; for each s:
//   dh_s = dOut[t(s)] + [s < T-1] (z_{s+1} * dh_{s+1} + W^T dgh_{s+1})
//   (dar, daz, dan) = dgi_s; dgh_s = (dar, daz, dan * r)
// doL: LN(R=1) of dOut; hL / savL: the forward's LN outputs (h_{s-1} is hL at step s-1, h0 at s=0);
// dgL: LN(R=4) of (dar, daz, dan, dan * r). dh0 [ndir][B][H] (optional) = W^T dgh_0 + z_0 * dh_0.
template <int H>
__global__ void __launch_bounds__(H * 2) gru16_bwd(const float* __restrict__ doL, const float* __restrict__ whh,
                                                   const float* __restrict__ hL, const float* __restrict__ savL,
                                                   const float* __restrict__ h0, float* __restrict__ dgL,
                                                   float* __restrict__ dh0, int B, int T, int ndir) {
  constexpr int G3 = 3 * H;
  constexpr int KR = 2 * H / 32;   // k-steps (gate rows) held in VGPRs: r and z gates
  constexpr int KN = H / 32;       // k-steps held in LDS: n gate
  constexpr int NW = H / 32;
  constexpr int GP = G3 + 8;       // bf16 row pitch of the dgh image
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16x8* wn_lds = reinterpret_cast<bf16x8*>(smem);                                // [NW][2][KN][64]
  uint16_t* gb = reinterpret_cast<uint16_t*>(smem + (size_t)NW * 2 * KN * 64 * 16);   // [BG][GP]

  const int d = blockIdx.y, bg = blockIdx.x, nbg = gridDim.x;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int lr = l & 15, lq = l >> 4;
  const float* W = whh + (int64_t)d * G3 * H;
  const int b = bg * BG + lr;
  const bool bok = b < B;

  // A = W^T: lane holds W[gate 32s + 8lq + j][unit (2w+ub)*16 + lr], j = 0..7
  bf16x8 wt[2][KR];
#pragma unroll
  for (int ub = 0; ub < 2; ++ub) {
    const int unit = (2 * w + ub) * 16 + lr;
#pragma unroll
    for (int s = 0; s < KR; ++s) wt[ub][s] = pack8_strided(W + (int64_t)(32 * s + 8 * lq) * H + unit, H);
#pragma unroll
    for (int s = 0; s < KN; ++s)
      wn_lds[((w * 2 + ub) * KN + s) * 64 + l] = pack8_strided(W + (int64_t)(2 * H + 32 * s + 8 * lq) * H + unit, H);
  }
  float dhn[2][4], zn[2][4];
#pragma unroll
  for (int ub = 0; ub < 2; ++ub)
#pragma unroll
    for (int i = 0; i < 4; ++i) dhn[ub][i] = zn[ub][i] = 0.f;
  __syncthreads();

  auto recur = [&](f32x4 (&acc)[2]) {
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) acc[ub] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint16_t* g0 = gb + lr * GP + 8 * lq;
    bf16x8 bf = *reinterpret_cast<const bf16x8*>(g0);
#pragma unroll
    for (int ks = 0; ks < KR + KN; ++ks) {
      bf16x8 bfn = bf;
      if (ks + 1 < KR + KN) bfn = *reinterpret_cast<const bf16x8*>(g0 + 32 * (ks + 1));
#pragma unroll
      for (int ub = 0; ub < 2; ++ub) {
        const bf16x8 a = ks < KR ? wt[ub][ks < KR ? ks : 0] : wn_lds[((w * 2 + ub) * KN + (ks - KR)) * 64 + l];
        acc[ub] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bf, acc[ub], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      bf = bfn;
    }
  };

  const uint32_t nbytes1 = (uint32_t)((int64_t)ndir * nbg * T * H * 16 * 4);
  const rsrc_t do_r = mkbuf(doL, nbytes1);
  const rsrc_t h_r = mkbuf(hL, nbytes1);
  const rsrc_t sv_r = mkbuf(savL, 4 * nbytes1);
  const rsrc_t dg_r = mkbuf(dgL, 4 * nbytes1);
  const rsrc_t h0_r = mkbuf(h0, (uint32_t)((int64_t)ndir * B * H * 4));   // null h0: loads return 0
  const uint32_t wb = (uint32_t)(2 * w) * 1024u, lo = (uint32_t)l * 16u, lane_b = wb + lo;
  const uint32_t h0_base = bok ? (uint32_t)(((int64_t)d * B + b) * H + (2 * w) * 16 + 4 * lq) * 4 : 0x80000000u;

  for (int s = T - 1; s >= 0; --s) {
    float4 dov[2], rv[2], zv[2], nv[2], gv[2], hv[2];
    const uint32_t od = ln_step(d, bg, nbg, T, s, H, 1) + lane_b;
    const uint32_t osv = ln_step(d, bg, nbg, T, s, H, 4) + 4 * wb + lo;
    const uint32_t ohp = ln_step(d, bg, nbg, T, s > 0 ? s - 1 : 0, H, 1) + lane_b;
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) {
      dov[ub] = bld4(do_r, od + (uint32_t)ub * 1024u);
      const uint32_t o = osv + (uint32_t)ub * 4096u;
      rv[ub] = bld4(sv_r, o);
      zv[ub] = bld4(sv_r, o + 1024u);
      nv[ub] = bld4(sv_r, o + 2048u);
      gv[ub] = bld4(sv_r, o + 3072u);
      hv[ub] = s > 0 ? bld4(h_r, ohp + (uint32_t)ub * 1024u) : bld4(h0_r, h0_base + (uint32_t)ub * 64u);
    }
    f32x4 acc[2];
    if (s < T - 1) recur(acc);
    else acc[0] = acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ar[2][4], az[2][4], an[2][4];
    const uint32_t og = ln_step(d, bg, nbg, T, s, H, 4) + 4 * wb + lo;
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float r = comp(rv[ub], i), z = comp(zv[ub], i), n = comp(nv[ub], i);
        const float dh = comp(dov[ub], i) + acc[ub][i] + zn[ub][i] * dhn[ub][i];
        const float dn = dh * (1.f - z);
        const float dz = dh * (comp(hv[ub], i) - n);
        const float dan = dn * (1.f - n * n);
        const float dr = dan * comp(gv[ub], i);
        ar[ub][i] = bok ? dr * r * (1.f - r) : 0.f;
        az[ub][i] = bok ? dz * z * (1.f - z) : 0.f;
        an[ub][i] = bok ? dan : 0.f;
        dhn[ub][i] = bok ? dh : 0.f;
        zn[ub][i] = z;
      }
      const uint32_t o = og + (uint32_t)ub * 4096u;
      const float4 a4 = make_float4(an[ub][0], an[ub][1], an[ub][2], an[ub][3]);
      bst4(dg_r, o, make_float4(ar[ub][0], ar[ub][1], ar[ub][2], ar[ub][3]));
      bst4(dg_r, o + 1024u, make_float4(az[ub][0], az[ub][1], az[ub][2], az[ub][3]));
      bst4(dg_r, o + 2048u, a4);
      bst4(dg_r, o + 3072u, mul4(a4, rv[ub]));
    }
    lds_barrier();   // every wave's MFMA reads of the previous dgh image are done
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) {
      const int j0 = (2 * w + ub) * 16 + 4 * lq;
      store_bf16x4(gb + lr * GP + j0, ar[ub][0], ar[ub][1], ar[ub][2], ar[ub][3]);
      store_bf16x4(gb + lr * GP + H + j0, az[ub][0], az[ub][1], az[ub][2], az[ub][3]);
      store_bf16x4(gb + lr * GP + 2 * H + j0, an[ub][0] * comp(rv[ub], 0), an[ub][1] * comp(rv[ub], 1),
                   an[ub][2] * comp(rv[ub], 2), an[ub][3] * comp(rv[ub], 3));
    }
    lds_barrier();
  }
  if (dh0) {
    f32x4 acc[2];
    recur(acc);
    if (bok) {
#pragma unroll
      for (int ub = 0; ub < 2; ++ub) {
        const int j0 = (2 * w + ub) * 16 + 4 * lq;
        *reinterpret_cast<float4*>(dh0 + ((int64_t)d * B + b) * H + j0) =
            make_float4(acc[ub][0] + zn[ub][0] * dhn[ub][0], acc[ub][1] + zn[ub][1] * dhn[ub][1],
                        acc[ub][2] + zn[ub][2] * dhn[ub][2], acc[ub][3] + zn[ub][3] * dhn[ub][3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------ layout permutation
// One thread per LN float4. to_lane: LN record k <- standard record rmap[k]; else standard record
// rmap[k] <- LN record k (k < Rl). Standard tensor (B, T, ndir*Rs*H); padded batch rows of the LN
// tensor are written as 0 (to_lane) or skipped.
__global__ void gru_lane_permute_k(const float* __restrict__ src, float* __restrict__ dst, int B, int T, int H,
                                   int ndir, int Rl, int Rs, unsigned rmap, int to_lane, int64_t n4) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n4) return;
  const int U = H / 16;
  const int nbg = (B + BG - 1) / BG;
  int64_t rest = idx;
  const int lane = (int)(rest % 64); rest /= 64;
  const int k = (int)(rest % Rl); rest /= Rl;
  const int ub = (int)(rest % U); rest /= U;
  const int s = (int)(rest % T); rest /= T;
  const int bg = (int)(rest % nbg);
  const int d = (int)(rest / nbg);
  const int b = bg * BG + (lane & 15);
  const int j = ub * 16 + 4 * (lane >> 4);
  const int t = d == 0 ? s : T - 1 - s;
  const int rs = (int)((rmap >> (4 * k)) & 15u);
  if (rs == 15) return;   // record not mapped
  const int64_t so = (((int64_t)b * T + t) * ndir + d) * Rs * H + (int64_t)rs * H + j;
  if (to_lane) {
    reinterpret_cast<float4*>(dst)[idx] =
        b < B ? *reinterpret_cast<const float4*>(src + so) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else if (b < B) {
    *reinterpret_cast<float4*>(dst + so) = reinterpret_cast<const float4*>(src)[idx];
  }
}

template <int H>
int launch_fwd(const float* giL, const float* whh, const float* bhh, const float* h0, float* hL, float* savL,
               int64_t B, int64_t T, int ndir, hipStream_t st) {
  static bool attr = false;
  const size_t shm = fwd_lds_bytes<H>();
  if (!attr) {
    B2P_CHECK_HIP(hipFuncSetAttribute((const void*)gru16_fwd<H>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr = true;
  }
  dim3 grid((unsigned)((B + BG - 1) / BG), (unsigned)ndir);
  hipLaunchKernelGGL(gru16_fwd<H>, grid, dim3(H * 2), shm, st, giL, whh, bhh, h0, hL, savL, (int)B, (int)T, ndir);
  B2P_CHECK_LAUNCH();
  return 0;
}

template <int H>
int launch_bwd(const float* doL, const float* whh, const float* hL, const float* savL, const float* h0, float* dgL,
               float* dh0, int64_t B, int64_t T, int ndir, hipStream_t st) {
  static bool attr = false;
  const size_t shm = bwd_lds_bytes<H>();
  if (!attr) {
    B2P_CHECK_HIP(hipFuncSetAttribute((const void*)gru16_bwd<H>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr = true;
  }
  dim3 grid((unsigned)((B + BG - 1) / BG), (unsigned)ndir);
  hipLaunchKernelGGL(gru16_bwd<H>, grid, dim3(H * 2), shm, st, doL, whh, hL, savL, h0, dgL, dh0, (int)B, (int)T,
                     ndir);
  B2P_CHECK_LAUNCH();
  return 0;
}
static_assert(fwd_lds_bytes<256>() <= 160 * 1024, "fwd LDS");
static_assert(bwd_lds_bytes<256>() <= 160 * 1024, "bwd LDS");

int ln_bytes_ok(int64_t B, int64_t T, int64_t H, int ndir, int R) {
  const int64_t nbg = (B + BG - 1) / BG;
  return ndir * nbg * BG * T * H * R * 4 < (int64_t)0x80000000LL;
}
}  // namespace

extern "C" int b2p_gru16_supported(int64_t H) { return H == 32 || H == 64 || H == 128 || H == 256; }

extern "C" int64_t b2p_gru16_lane_floats(int64_t B, int64_t T, int64_t H, int ndir, int R) {
  return (int64_t)ndir * ((B + BG - 1) / BG) * BG * T * H * R;
}

extern "C" int b2p_gru_lane_permute(const float* src, float* dst, int64_t B, int64_t T, int64_t H, int ndir, int Rl,
                                    int Rs, uint32_t rmap, int to_lane, b2p_stream_t stream) {
  B2P_CHECK_ARG(src && dst, "gru_lane_permute: NULL pointer");
  B2P_CHECK_ARG(H % 16 == 0 && Rl >= 1 && Rl <= 8 && Rs >= 1 && Rs <= 14, "gru_lane_permute: bad shape");
  const int64_t n4 = b2p_gru16_lane_floats(B, T, H, ndir, Rl) / 4;
  if (n4 <= 0) return 0;
  hipLaunchKernelGGL(gru_lane_permute_k, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, src,
                     dst, (int)B, (int)T, (int)H, ndir, Rl, Rs, rmap, to_lane, n4);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_gru_fwd16(const float* giL, const float* whh, const float* bhh, const float* h0, float* hL,
                             float* savL, int64_t B, int64_t T, int64_t H, int ndir, b2p_stream_t stream) {
  B2P_CHECK_ARG(giL && whh && hL && savL, "gru_fwd16: NULL pointer");
  B2P_CHECK_ARG(b2p_gru16_supported(H), "gru_fwd16: hidden size %lld unsupported (32, 64, 128 or 256)", (long long)H);
  B2P_CHECK_ARG(ndir == 1 || ndir == 2, "gru_fwd16: ndir must be 1 or 2");
  B2P_CHECK_ARG(ln_bytes_ok(B, T, H, ndir, 4), "gru_fwd16: lane-native buffers exceed 2 GiB");
  if (B <= 0 || T <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (H == 32) return launch_fwd<32>(giL, whh, bhh, h0, hL, savL, B, T, ndir, st);
  if (H == 64) return launch_fwd<64>(giL, whh, bhh, h0, hL, savL, B, T, ndir, st);
  if (H == 128) return launch_fwd<128>(giL, whh, bhh, h0, hL, savL, B, T, ndir, st);
  return launch_fwd<256>(giL, whh, bhh, h0, hL, savL, B, T, ndir, st);
}

extern "C" int b2p_gru_bwd16(const float* doL, const float* whh, const float* hL, const float* savL, const float* h0,
                             float* dgL, float* dh0, int64_t B, int64_t T, int64_t H, int ndir, b2p_stream_t stream) {
  B2P_CHECK_ARG(doL && whh && hL && savL && dgL, "gru_bwd16: NULL pointer");
  B2P_CHECK_ARG(b2p_gru16_supported(H), "gru_bwd16: hidden size %lld unsupported (32, 64, 128 or 256)", (long long)H);
  B2P_CHECK_ARG(ndir == 1 || ndir == 2, "gru_bwd16: ndir must be 1 or 2");
  B2P_CHECK_ARG(ln_bytes_ok(B, T, H, ndir, 4), "gru_bwd16: lane-native buffers exceed 2 GiB");
  if (B <= 0 || T <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (H == 32) return launch_bwd<32>(doL, whh, hL, savL, h0, dgL, dh0, B, T, ndir, st);
  if (H == 64) return launch_bwd<64>(doL, whh, hL, savL, h0, dgL, dh0, B, T, ndir, st);
  if (H == 128) return launch_bwd<128>(doL, whh, hL, savL, h0, dgL, dh0, B, T, ndir, st);
  return launch_bwd<256>(doL, whh, hL, savL, h0, dgL, dh0, B, T, ndir, st);
}
