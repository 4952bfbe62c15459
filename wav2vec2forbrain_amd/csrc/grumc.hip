// Multi-CU persistent GRU recurrence (nn.GRU semantics, gate order r, z, n) for hidden sizes too
// large for one CU (the Conformer experiment's brain encoder: H = 512 x 3 layers, reference
// src/model/brain_feature_extractor.py:39-47, 56-68; README encoder H512x3), bf16 precision mode.
//
// One launch runs the whole time loop. A recurrence (direction d, 16 batch rows) is spread over
// P = H/64 workgroups ("members"), one per CU: member m owns hidden units [64m, 64m+64) and keeps
// their W_hh rows (r, z, n: 192 x H; fp16 in the forward, bf16 in the backward) in registers as MFMA
// A-fragments for the whole launch, so W_hh is read from HBM once per launch instead of once per
// step. Per step the members exchange the new state through L2 as tagged 8-byte granules ({tag =
// step+1, two fp16 h values / three bf16 dgh values}: written by one sc1
// store, polled by sc1 loads until every tag matches; MI355X_MICROARCH.md 'Workgroup dispatch, XCD
// placement & inter-workgroup visibility', cdna_hip_programming.md Guideline 16 R2) — no fences,
// no flags, no grid barrier. The exchange slots are zeroed by a memset before every launch (so tags
// of a previous launch or graph replay never match) and double-buffered by step parity (a member
// can be at most one step ahead of any other). Workgroups of one recurrence take block ids with
// equal blockIdx % 8 (one XCD under the observed round-robin placement: speed only).
//
//   forward : gates^T (3 x 64 x 16) = W_hh[rows of m] (192 x H) . h_{t-1}^T (H x 16), fp32 acc
//   backward: dh_rec^T (64 x 16)    = W_hh[:, units of m]^T (64 x 3H) . dgh_{t+1}^T (3H x 16)
// Inputs / outputs use the standard layouts of the per-step kernels (csrc/gru.hip), so these are
// drop-in for b2p_gru_fwd / b2p_gru_bwd: gi, dgi, dgh [B][T][ndir*3H], out [B][T][ndir*H],
// saved [B][T][ndir][4][H] = (r, z, n, W_hn h + b_hn), h0 / dh0 [ndir][B][H].
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {
constexpr int BG = 16;        // batch rows per recurrence (MFMA N)
constexpr int UPM = 64;       // hidden units per member
constexpr int NTH = 256;      // 4 waves x 16 units
constexpr unsigned SPIN_MAX = 1u << 22;
constexpr int IDS_PER_GROUP = 16;   // members' XCC ids (P <= 16)
constexpr int MAX_GROUPS = 32;      // (direction, 16-row batch group) recurrences per launch
constexpr int64_t HDR_BYTES = 16 + (int64_t)MAX_GROUPS * IDS_PER_GROUP * 8;   // fail word + ids

typedef __attribute__((address_space(1))) unsigned long long gu64;

// Granule stores: sc1 (write-through to memory: visible to any XCD) or, when every member of the
// recurrence runs on this XCD (checked at launch, see same_xcd), a workgroup-scope store (sc0: the
// line stays in the XCD's L2, where the other members' sc1 loads read it, ~2x closer than memory).
__device__ __forceinline__ void store_granule(unsigned long long* p, unsigned long long x, bool local) {
  if (local)
    __hip_atomic_store((gu64*)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    __hip_atomic_store((gu64*)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void put_granule(unsigned long long* p, unsigned tag, unsigned v, bool local) {
  store_granule(p, ((unsigned long long)tag << 32) | v, local);
}
__device__ __forceinline__ unsigned long long get_granule(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return (unsigned)b2p_bf16_bits(a) | ((unsigned)b2p_bf16_bits(b) << 16);
}
__device__ __forceinline__ unsigned pack2h(float a, float b) {
  return (unsigned)b2p_f16_bits(a) | ((unsigned)b2p_f16_bits(b) << 16);
}
__device__ __forceinline__ bf16x8 pack8_strided(const float* p, int64_t stride) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)p[j * stride];
  return r;
}
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)); }
__device__ __forceinline__ float4 f4(const f32x4& a) { return make_float4(a[0], a[1], a[2], a[3]); }

// Sweep N granules per lane (stride NTH, starting at this lane) until every tag == tag; the values
// go to u32 LDS words at dst(q). On timeout the kernel records `fail` and stops waiting (the results
// are then garbage, the launch still terminates); the caller folds `fail` into a persistent status
// word right after the launch (b2p_gru_mc_status), which the host checks at its next sync and raises.
template <int N, typename Tag, typename Dst>
__device__ __forceinline__ void sweep(const unsigned long long* slot, Tag tag_ok, Dst dst, int* fail, bool& dead) {
  static_assert(N <= 64, "one 64-bit pending mask per lane");
  const int lane = threadIdx.x;
  unsigned long long v[N];
  unsigned long long miss = 0;   // granules of this lane not yet seen with this step's tag
#pragma unroll
  for (int k = 0; k < N; ++k) {
    v[k] = get_granule(slot + k * NTH + lane);
    if (!tag_ok(v[k])) miss |= 1ull << k;
  }
  for (unsigned spins = 0; __any(miss != 0) && !dead; ++spins) {
    if (spins > SPIN_MAX) {
      dead = true;
      if (lane == 0) __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (miss & (1ull << k)) {
        v[k] = get_granule(slot + k * NTH + lane);
        if (tag_ok(v[k])) miss &= ~(1ull << k);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < N; ++k) dst(k * NTH + lane, v[k]);
}

// recurrence (d, bg) and member of this block; false for blocks with no work
__device__ __forceinline__ bool place(int P, int ngroups, int& d, int& bg, int& m, int nbg) {
  int g;
  if (ngroups <= 8) {   // members of a group on blocks with equal blockIdx % 8
    g = blockIdx.x % 8;
    m = blockIdx.x / 8;
    if (g >= ngroups) return false;
  } else {
    g = blockIdx.x % ngroups;
    m = blockIdx.x / ngroups;
  }
  d = g / nbg;
  bg = g % nbg;
  return m < P;
}

// Are all P members of this recurrence on one XCD? Each member publishes its XCC id once (sc1), every
// member reads all of them; the answer is uniform across the group, so the group agrees on the store
// flavour of every later granule. Placement is never assumed: any member elsewhere -> sc1 stores.
__device__ __forceinline__ bool same_xcd(unsigned long long* ids, int P, int m, int* fail, bool& dead) {
  __shared__ int all_same;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 0xFu;
  if (threadIdx.x == 0) {
    __hip_atomic_store((gu64*)(ids + m), (1ull << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    all_same = 1;
  }
  __syncthreads();
  if (threadIdx.x < 64) {   // one wave polls the P ids
    unsigned long long x = 0;
    bool ok = threadIdx.x >= P;
    for (unsigned spins = 0; !__all(ok); ++spins) {
      if (spins > SPIN_MAX) {
        dead = true;
        if (threadIdx.x == 0) __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (!ok) {
        x = get_granule(ids + threadIdx.x);
        ok = (unsigned)(x >> 32) == 1u;
      }
    }
    if (threadIdx.x < P && (unsigned)x != xcc) all_same = 0;
  }
  __syncthreads();
  const bool same = all_same != 0 && !dead;
  if (same && m == 0 && threadIdx.x == 0) atomicAdd(fail + 1, 1);   // diagnostic: groups on one XCD
  return same;
}

// ------------------------------------------------------------------------------------------ forward
// exchange slots: [group][2][P * 512] granules (h_s of member m, batch b, unit pair p at
// m*512 + b*32 + p)
template <int H>
__global__ void __launch_bounds__(NTH, 1) grumc_fwd(const float* __restrict__ gi, const float* __restrict__ whh,
                                                    const float* __restrict__ bhh, const float* __restrict__ h0,
                                                    float* __restrict__ out, float* __restrict__ saved,
                                                    unsigned long long* xch, unsigned long long* ids, int* fail, int B,
                                                    int T, int ndir, int nbg, int withhold) {
  constexpr int P = H / UPM;
  constexpr int KS = H / 32;
  constexpr int HPW = H / 2 + 4;              // u32 words per batch row of the h image (16-B stagger)
  constexpr int NGR = P * 512 / NTH;          // granules swept per lane
  constexpr int G3 = 3 * H;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned* hw = reinterpret_cast<unsigned*>(smem);   // [2][BG][HPW] u32 (fp16 pairs)

  int d, bg, m;
  if (!place(P, ndir * nbg, d, bg, m, nbg)) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lq = l >> 4;
  const int b = bg * BG + lr;
  const bool bok = b < B;
  const int u0 = m * UPM + w * 16;             // first unit of this wave's block
  const int j0 = u0 + 4 * lq;                  // this lane's 4 output units
  const float* W = whh + (int64_t)d * G3 * H;
  unsigned long long* xg = xch + (int64_t)(d * nbg + bg) * 2 * P * 512;
  bool dead = false;
  const bool local = same_xcd(ids + (d * nbg + bg) * IDS_PER_GROUP, P, m, fail, dead);

  bf16x8 wf[3][KS];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int s = 0; s < KS; ++s) wf[g][s] = b2p_pack8_f16(W + (int64_t)(g * H + u0 + lr) * H + 32 * s + 8 * lq);
  float4 bh[3];
#pragma unroll
  for (int g = 0; g < 3; ++g)
    bh[g] = bhh ? *reinterpret_cast<const float4*>(bhh + (int64_t)d * G3 + g * H + j0) : make_float4(0.f, 0.f, 0.f, 0.f);

  // h_{-1}: h0 (or zeros) straight into image 0, and this lane's own 4 values in registers
  float hp[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = tid; i < BG * (H / 2); i += NTH) {
    const int r = i / (H / 2), c = i % (H / 2);
    const int bb = bg * BG + r;
    float a = 0.f, c2 = 0.f;
    if (h0 && bb < B) {
      a = h0[((int64_t)d * B + bb) * H + 2 * c];
      c2 = h0[((int64_t)d * B + bb) * H + 2 * c + 1];
    }
    hw[r * HPW + c] = pack2h(a, c2);
  }
  if (h0 && bok) {
    const float4 v = *reinterpret_cast<const float4*>(h0 + ((int64_t)d * B + b) * H + j0);
    hp[0] = v.x; hp[1] = v.y; hp[2] = v.z; hp[3] = v.w;
  }
  __syncthreads();

  const int64_t gstride = (int64_t)ndir * G3, ostride = (int64_t)ndir * H;
  // vmcnt counts loads and stores together, in issue order, so the granule stores go out first in a
  // step; the outputs and the next step's input loads follow and complete while the other members
  // are still on their way to the next exchange.
  auto load_gi = [&](int s, float4 (&g)[3]) {
    const int t = d == 0 ? s : T - 1 - s;
    const float* gp = gi + ((int64_t)b * T + t) * gstride + d * G3 + j0;
    if (bok)
#pragma unroll
      for (int q = 0; q < 3; ++q) g[q] = *reinterpret_cast<const float4*>(gp + q * H);
  };
  float4 gc[3];   // this step's input projection (the next step's is loaded into it once consumed)
#pragma unroll
  for (int q = 0; q < 3; ++q) gc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  load_gi(0, gc);
  float st_h[4], st_r[4], st_z[4], st_n[4], st_g[4];   // this step's outputs
  auto store_out = [&](int s) {
    if (!bok) return;
    const int t = d == 0 ? s : T - 1 - s;
    *reinterpret_cast<float4*>(out + ((int64_t)b * T + t) * ostride + d * H + j0) =
        make_float4(st_h[0], st_h[1], st_h[2], st_h[3]);
    float* sv = saved + (((int64_t)b * T + t) * ndir + d) * 4 * H + j0;
    *reinterpret_cast<float4*>(sv) = make_float4(st_r[0], st_r[1], st_r[2], st_r[3]);
    *reinterpret_cast<float4*>(sv + H) = make_float4(st_z[0], st_z[1], st_z[2], st_z[3]);
    *reinterpret_cast<float4*>(sv + 2 * H) = make_float4(st_n[0], st_n[1], st_n[2], st_n[3]);
    *reinterpret_cast<float4*>(sv + 3 * H) = make_float4(st_g[0], st_g[1], st_g[2], st_g[3]);
  };
  for (int s = 0; s < T; ++s) {
    float4 (&g)[3] = gc;
    if (s > 0) {   // h_{s-1} of every member: tags s, slot (s-1) & 1 -> image s & 1
      unsigned* img = hw + (s & 1) * BG * HPW;
      const unsigned tag = (unsigned)s;
      sweep<NGR>(xg + ((s - 1) & 1) * P * 512, [tag](unsigned long long x) { return (unsigned)(x >> 32) == tag; },
                 [&](int q, unsigned long long x) { img[((q >> 5) & 15) * HPW + (q >> 9) * 32 + (q & 31)] = (unsigned)x; },
                 fail, dead);
      __syncthreads();
    }
    // gate pre-activations: acc = gi + b_hh (r, z) / b_hn (n) + W . h
    f32x4 acc[3];
    acc[0] = f32x4{g[0].x + bh[0].x, g[0].y + bh[0].y, g[0].z + bh[0].z, g[0].w + bh[0].w};
    acc[1] = f32x4{g[1].x + bh[1].x, g[1].y + bh[1].y, g[1].z + bh[1].z, g[1].w + bh[1].w};
    acc[2] = f32x4{bh[2].x, bh[2].y, bh[2].z, bh[2].w};
    const unsigned* hrow = hw + (s & 1) * BG * HPW + lr * HPW + 4 * lq;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 bf = *reinterpret_cast<const bf16x8*>(hrow + 16 * ks);
#pragma unroll
      for (int q = 0; q < 3; ++q) acc[q] = b2p_mfma_f16(wf[q][ks], bf, acc[q]);
    }
    const float gnv[4] = {g[2].x, g[2].y, g[2].z, g[2].w};
    float hh[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float rr = sigm(acc[0][i]);
      const float zz = sigm(acc[1][i]);
      const float nn = tanh_fast(gnv[i] + rr * acc[2][i]);
      hh[i] = bok ? (1.f - zz) * nn + zz * hp[i] : 0.f;
      hp[i] = hh[i];
      st_h[i] = hh[i];
      st_r[i] = rr;
      st_z[i] = zz;
      st_n[i] = nn;
      st_g[i] = acc[2][i];
    }
    // publish h_s (fp16 pairs) FIRST: the other members wait on it, and a later store or load issued
    // before it would delay it; then this step's outputs and the next step's input projection
    if (s + 1 < T && m != withhold) {   // withhold: test knob (b2p_gru_mc_debug_withhold), -1 = off
      unsigned long long* dst = xg + (s & 1) * P * 512 + m * 512 + lr * 32 + w * 8 + lq * 2;
      put_granule(dst, (unsigned)(s + 1), pack2h(hh[0], hh[1]), local);
      put_granule(dst + 1, (unsigned)(s + 1), pack2h(hh[2], hh[3]), local);
    }
    store_out(s);
    if (s + 1 < T) load_gi(s + 1, gc);
  }
}

// ----------------------------------------------------------------------------------------- backward
// Processing steps run backwards (s = T-1 .. 0, t = t(s)). For own units j:
//   dh_s = dout[t] + [s < T-1] (z_{s+1} dh_{s+1} + (W^T dgh_{s+1})_j)
//   dn = dh (1-z); dz = dh (h_{s-1} - n); dan = dn (1 - n^2); dar = dan ghn r (1-r); daz = dz z (1-z)
//   dgi = (dar, daz, dan), dgh = (dar, daz, dan r)
// The reduction runs over all 3H gate rows in the interleaved order k = 3*unit + gate, so one unit's
// three dgh values travel in ONE granule {bf16 r, bf16 z | bf16 n, 16-bit tag} and land as three
// consecutive bf16 of the LDS image; W^T's A-fragments are gathered in the same order.
// exchange slots: [group][2][P * 1024] granules (member m, batch b, unit u of m at m*1024 + b*64 + u)
__device__ __forceinline__ unsigned long long dgh_granule(float r, float z, float n, unsigned tag) {
  return (unsigned long long)pack2(r, z) | ((unsigned long long)(b2p_bf16_bits(n) | (tag << 16)) << 32);
}

template <int H>
__global__ void __launch_bounds__(NTH, 1) grumc_bwd(const float* __restrict__ dout, const float* __restrict__ whh,
                                                    const float* __restrict__ out, const float* __restrict__ saved,
                                                    const float* __restrict__ h0, float* __restrict__ dgi,
                                                    float* __restrict__ dgh, float* __restrict__ dh0,
                                                    unsigned long long* xch, unsigned long long* ids, int* fail, int B,
                                                    int T, int ndir, int nbg, int withhold) {
  constexpr int P = H / UPM;
  constexpr int G3 = 3 * H;
  constexpr int KS = G3 / 32;                  // k-steps over all gate rows
  constexpr int GPH = G3 + 8;                  // bf16 per batch row of the dgh image (16-B stagger)
  constexpr int NGR = P * 1024 / NTH;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* gimg = reinterpret_cast<uint16_t*>(smem);   // [2][BG][GPH] bf16, k = 3*unit + gate

  int d, bg, m;
  if (!place(P, ndir * nbg, d, bg, m, nbg)) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lq = l >> 4;
  const int b = bg * BG + lr;
  const bool bok = b < B;
  const int u0 = m * UPM + w * 16;
  const int j0 = u0 + 4 * lq;
  const float* W = whh + (int64_t)d * G3 * H;
  unsigned long long* xg = xch + (int64_t)(d * nbg + bg) * 2 * P * 1024;
  bool dead = false;
  const bool local = same_xcd(ids + (d * nbg + bg) * IDS_PER_GROUP, P, m, fail, dead);

  // A = W^T in the interleaved k order: lane holds W[gate(k)*H + unit(k)][u0 + lr], k = 32s + 8lq + i
  bf16x8 wt[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = 32 * s + 8 * lq + i;
      wt[s][i] = (__bf16)W[(int64_t)((k % 3) * H + k / 3) * H + u0 + lr];
    }
  }

  float dhn[4] = {0.f, 0.f, 0.f, 0.f}, zn[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t gstride = (int64_t)ndir * G3, ostride = (int64_t)ndir * H;
  // as in the forward: granules first, then this step's outputs, then the next step's inputs
  auto load_in = [&](int s, float4 (&v)[6]) __attribute__((always_inline)) {   // dout, r, z, n, ghn, h_{s-1}
    if (!bok) return;
    const int t = d == 0 ? s : T - 1 - s;
    const int tp = d == 0 ? t - 1 : t + 1;
    v[0] = *reinterpret_cast<const float4*>(dout + ((int64_t)b * T + t) * ostride + d * H + j0);
    const float* sv = saved + (((int64_t)b * T + t) * ndir + d) * 4 * H + j0;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[1 + q] = *reinterpret_cast<const float4*>(sv + q * H);
    if (s > 0) v[5] = *reinterpret_cast<const float4*>(out + ((int64_t)b * T + tp) * ostride + d * H + j0);
    else if (h0) v[5] = *reinterpret_cast<const float4*>(h0 + ((int64_t)d * B + b) * H + j0);
    else v[5] = make_float4(0.f, 0.f, 0.f, 0.f);   // h_{-1} = 0 (the buffer still holds step 1's h_0)
  };
  float4 ic[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) ic[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  load_in(T - 1, ic);
  float st_ar[4], st_az[4], st_an[4], st_r[4];   // this step's outputs
  auto store_out = [&](int s) __attribute__((always_inline)) {
    if (!bok) return;
    const int t = d == 0 ? s : T - 1 - s;
    float* gp = dgi + ((int64_t)b * T + t) * gstride + d * G3 + j0;
    float* hq = dgh + ((int64_t)b * T + t) * gstride + d * G3 + j0;
    const float4 a4 = make_float4(st_ar[0], st_ar[1], st_ar[2], st_ar[3]);
    const float4 z4 = make_float4(st_az[0], st_az[1], st_az[2], st_az[3]);
    *reinterpret_cast<float4*>(gp) = a4;
    *reinterpret_cast<float4*>(gp + H) = z4;
    *reinterpret_cast<float4*>(gp + 2 * H) = make_float4(st_an[0], st_an[1], st_an[2], st_an[3]);
    *reinterpret_cast<float4*>(hq) = a4;
    *reinterpret_cast<float4*>(hq + H) = z4;
    *reinterpret_cast<float4*>(hq + 2 * H) = make_float4(st_an[0] * st_r[0], st_an[1] * st_r[1], st_an[2] * st_r[2],
                                                         st_an[3] * st_r[3]);
  };
  // W^T . dgh_{s+1} from the exchange (tag s+2, slot (s+1) & 1 -> image (s+1) & 1)
  auto recur = [&](int s) __attribute__((always_inline)) {
    uint16_t* img = gimg + ((s + 1) & 1) * BG * GPH;
    const unsigned tag = (unsigned)(s + 2);
    sweep<NGR>(xg + ((s + 1) & 1) * P * 1024, [tag](unsigned long long x) { return (unsigned)(x >> 48) == tag; },
               [&](int q, unsigned long long x) {
                 const int mm = q >> 10, bb = (q >> 6) & 15, u = q & 63;
                 const int k = 3 * (mm * UPM + u);
                 uint16_t* p = img + bb * GPH + k;
                 const unsigned lo = (unsigned)x, n = (unsigned)(x >> 32) & 0xFFFFu;
                 if (k & 1) {          // r at an odd position: r, then (z, n) as one aligned word
                   p[0] = (uint16_t)lo;
                   *reinterpret_cast<unsigned*>(p + 1) = (lo >> 16) | (n << 16);
                 } else {              // (r, z) as one aligned word, then n
                   *reinterpret_cast<unsigned*>(p) = lo;
                   p[2] = (uint16_t)n;
                 }
               }, fail, dead);
    __syncthreads();
    // two independent accumulation chains (even / odd k-steps): the MFMA pipe never waits on the
    // previous MFMA's result
    f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
    const uint16_t* grow = img + lr * GPH + 8 * lq;
#pragma unroll
    for (int ks = 0; ks < KS; ks += 2) {
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(grow + 32 * ks);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(grow + 32 * (ks + 1));
      a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt[ks], b0, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt[ks + 1], b1, a1, 0, 0, 0);
    }
    return f32x4{a0[0] + a1[0], a0[1] + a1[1], a0[2] + a1[2], a0[3] + a1[3]};
  };
  // one input buffer: step s-1's inputs are loaded once step s has consumed them (behind the publish,
  // so they overlap the other members' arrival)
  for (int s = T - 1; s >= 0; --s) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s < T - 1) acc = recur(s);
    const float dv[4] = {ic[0].x, ic[0].y, ic[0].z, ic[0].w}, r4[4] = {ic[1].x, ic[1].y, ic[1].z, ic[1].w};
    const float z4[4] = {ic[2].x, ic[2].y, ic[2].z, ic[2].w}, n4[4] = {ic[3].x, ic[3].y, ic[3].z, ic[3].w};
    const float g4[4] = {ic[4].x, ic[4].y, ic[4].z, ic[4].w}, h4[4] = {ic[5].x, ic[5].y, ic[5].z, ic[5].w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dh = dv[i] + (s < T - 1 ? acc[i] + zn[i] * dhn[i] : 0.f);
      const float dn = dh * (1.f - z4[i]);
      const float dz = dh * (h4[i] - n4[i]);
      const float dan = dn * (1.f - n4[i] * n4[i]);
      st_ar[i] = bok ? dan * g4[i] * r4[i] * (1.f - r4[i]) : 0.f;
      st_az[i] = bok ? dz * z4[i] * (1.f - z4[i]) : 0.f;
      st_an[i] = bok ? dan : 0.f;
      st_r[i] = r4[i];
      dhn[i] = bok ? dh : 0.f;
      zn[i] = z4[i];
    }
    if ((s > 0 || dh0) && m != withhold) {   // the step before (or dh0) needs this step's dgh
      unsigned long long* dst = xg + (s & 1) * P * 1024 + m * 1024 + lr * 64 + w * 16 + lq * 4;
      const unsigned tag = (unsigned)(s + 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        store_granule(dst + i, dgh_granule(st_ar[i], st_az[i], st_an[i] * st_r[i], tag), local);
    }
    store_out(s);
    if (s > 0) load_in(s - 1, ic);
  }
  if (dh0) {   // dh0 = W^T dgh_0 + z_0 dh_0
    const f32x4 acc = recur(-1);
    if (bok)
      *reinterpret_cast<float4*>(dh0 + ((int64_t)d * B + b) * H + j0) =
          make_float4(acc[0] + zn[0] * dhn[0], acc[1] + zn[1] * dhn[1], acc[2] + zn[2] * dhn[2], acc[3] + zn[3] * dhn[3]);
  }
}

template <int H>
constexpr size_t fwd_lds() { return (size_t)2 * BG * (H / 2 + 4) * 4; }
template <int H>
constexpr size_t bwd_lds() { return (size_t)2 * BG * (3 * H + 8) * 2; }

int grid_blocks(int P, int ngroups) { return ngroups <= 8 ? 8 * P : ngroups * P; }

// test knob (b2p_gru_mc_debug_withhold): this member skips its granule stores, so the others time out
int g_withhold = -1;

template <int H>
int launch_fwd(const float* gi, const float* whh, const float* bhh, const float* h0, float* out, float* saved,
               unsigned long long* xch, unsigned long long* ids, int* fail, int B, int T, int ndir, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    B2P_CHECK_HIP(hipFuncSetAttribute((const void*)grumc_fwd<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)fwd_lds<H>()));
    attr = true;
  }
  const int nbg = (B + BG - 1) / BG;
  hipLaunchKernelGGL(grumc_fwd<H>, dim3(grid_blocks(H / UPM, ndir * nbg)), dim3(NTH), fwd_lds<H>(), st, gi, whh, bhh,
                     h0, out, saved, xch, ids, fail, B, T, ndir, nbg, g_withhold);
  B2P_CHECK_LAUNCH();
  return 0;
}

template <int H>
int launch_bwd(const float* dout, const float* whh, const float* out, const float* saved, const float* h0, float* dgi,
               float* dgh, float* dh0, unsigned long long* xch, unsigned long long* ids, int* fail, int B, int T,
               int ndir, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    B2P_CHECK_HIP(hipFuncSetAttribute((const void*)grumc_bwd<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)bwd_lds<H>()));
    attr = true;
  }
  const int nbg = (B + BG - 1) / BG;
  hipLaunchKernelGGL(grumc_bwd<H>, dim3(grid_blocks(H / UPM, ndir * nbg)), dim3(NTH), bwd_lds<H>(), st, dout, whh,
                     out, saved, h0, dgi, dgh, dh0, xch, ids, fail, B, T, ndir, nbg, g_withhold);
  B2P_CHECK_LAUNCH();
  return 0;
}

bool mc_supported(int64_t H) { return H == 256 || H == 384 || H == 512; }

__global__ void zero16_k(uint4* __restrict__ p, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}

__global__ void mc_status_k(const int* __restrict__ fail, int32_t* status, int32_t code) {
  if (threadIdx.x == 0 && fail[0] != 0) atomicCAS(status, 0, code);
}
}  // namespace

extern "C" int b2p_gru_mc_supported(int64_t H) { return mc_supported(H) ? 1 : 0; }

extern "C" int b2p_gru_mc_status(const void* workspace, int32_t* status, int32_t code, b2p_stream_t stream) {
  B2P_CHECK_ARG(workspace && status, "gru_mc_status: NULL pointer");
  B2P_CHECK_ARG(code != 0, "gru_mc_status: code must be nonzero");
  hipLaunchKernelGGL(mc_status_k, dim3(1), dim3(64), 0, (hipStream_t)stream, (const int*)workspace, status, code);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_gru_mc_debug_withhold(int member) {
  B2P_CHECK_ARG(member >= -1 && member < 16, "gru_mc_debug_withhold: member must be -1 (off) or 0..15");
  g_withhold = member;
  return 0;
}

// exchange buffer (bytes, before the 16-B-aligned fail word block): 2 slots x granules per group
extern "C" int64_t b2p_gru_mc_workspace(int64_t B, int64_t H, int ndir) {
  if (!mc_supported(H)) return 0;
  const int64_t nbg = (B + BG - 1) / BG, P = H / UPM;
  return HDR_BYTES + (int64_t)ndir * nbg * 2 * P * 1024 * 8;   // sized for the backward (2x the forward)
}

static int mc_prepare(void* ws, int64_t B, int64_t H, int ndir, hipStream_t st, unsigned long long** xch,
                      unsigned long long** ids, int** fail) {
  const int64_t bytes = b2p_gru_mc_workspace(B, H, ndir);
  // every polled word (tags) and the fail flag are zeroed before every launch, by a kernel (a node of
  // a captured graph, replayed first): granules of a previous launch never match this launch's tags.
  // (A captured hipMemsetAsync node was observed leaving foreign bytes in the first 16 bytes of the
  // block on replays after the first, ROCm 7.2.)
  const int64_t n16 = bytes / 16;
  const int64_t nb = (n16 + 255) / 256;
  hipLaunchKernelGGL(zero16_k, dim3((unsigned)(nb < 1024 ? nb : 1024)), dim3(256), 0, st, (uint4*)ws, n16);
  B2P_CHECK_LAUNCH();
  *fail = reinterpret_cast<int*>(ws);
  *ids = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws) + 16);
  *xch = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ws) + HDR_BYTES);
  return 0;
}

extern "C" int b2p_gru_fwd_mc(const float* gi, const float* whh, const float* bhh, const float* h0, float* out,
                              float* saved, void* workspace, int64_t B, int64_t T, int64_t H, int ndir,
                              b2p_stream_t stream) {
  B2P_CHECK_ARG(gi && whh && out && saved && workspace, "gru_fwd_mc: NULL pointer");
  B2P_CHECK_ARG(mc_supported(H), "gru_fwd_mc: hidden size %lld unsupported (256, 384 or 512)", (long long)H);
  B2P_CHECK_ARG(ndir == 1 || ndir == 2, "gru_fwd_mc: ndir must be 1 or 2");
  B2P_CHECK_ARG((((uintptr_t)workspace) & 15u) == 0, "gru_fwd_mc: workspace must be 16-byte aligned");
  if (B <= 0 || T <= 0) return 0;
  const int nbg = (int)((B + BG - 1) / BG);
  B2P_CHECK_ARG(grid_blocks((int)(H / UPM), ndir * nbg) <= 256 && ndir * nbg <= MAX_GROUPS,
                "gru_fwd_mc: more recurrences than CUs");
  hipStream_t st = (hipStream_t)stream;
  unsigned long long *xch, *ids;
  int* fail;
  if (mc_prepare(workspace, B, H, ndir, st, &xch, &ids, &fail)) return 2;
  if (H == 256) return launch_fwd<256>(gi, whh, bhh, h0, out, saved, xch, ids, fail, (int)B, (int)T, ndir, st);
  if (H == 384) return launch_fwd<384>(gi, whh, bhh, h0, out, saved, xch, ids, fail, (int)B, (int)T, ndir, st);
  return launch_fwd<512>(gi, whh, bhh, h0, out, saved, xch, ids, fail, (int)B, (int)T, ndir, st);
}

extern "C" int b2p_gru_bwd_mc(const float* dout, const float* whh, const float* out, const float* saved,
                              const float* h0, float* dgi, float* dgh, float* dh0, void* workspace, int64_t B,
                              int64_t T, int64_t H, int ndir, b2p_stream_t stream) {
  B2P_CHECK_ARG(dout && whh && out && saved && dgi && dgh && workspace, "gru_bwd_mc: NULL pointer");
  B2P_CHECK_ARG(mc_supported(H), "gru_bwd_mc: hidden size %lld unsupported (256, 384 or 512)", (long long)H);
  B2P_CHECK_ARG(ndir == 1 || ndir == 2, "gru_bwd_mc: ndir must be 1 or 2");
  B2P_CHECK_ARG((((uintptr_t)workspace) & 15u) == 0, "gru_bwd_mc: workspace must be 16-byte aligned");
  if (B <= 0 || T <= 0) return 0;
  const int nbg = (int)((B + BG - 1) / BG);
  B2P_CHECK_ARG(grid_blocks((int)(H / UPM), ndir * nbg) <= 256 && ndir * nbg <= MAX_GROUPS,
                "gru_bwd_mc: more recurrences than CUs");
  // the backward granule carries a 16-bit step tag (dgh_granule): tags 1..T must stay distinct
  B2P_CHECK_ARG(T + 1 <= 0xFFFF, "gru_bwd_mc: T = %lld exceeds the 16-bit step tag", (long long)T);
  hipStream_t st = (hipStream_t)stream;
  unsigned long long *xch, *ids;
  int* fail;
  if (mc_prepare(workspace, B, H, ndir, st, &xch, &ids, &fail)) return 2;
  if (H == 256)
    return launch_bwd<256>(dout, whh, out, saved, h0, dgi, dgh, dh0, xch, ids, fail, (int)B, (int)T, ndir, st);
  if (H == 384)
    return launch_bwd<384>(dout, whh, out, saved, h0, dgi, dgh, dh0, xch, ids, fail, (int)B, (int)T, ndir, st);
  return launch_bwd<512>(dout, whh, out, saved, h0, dgi, dgh, dh0, xch, ids, fail, (int)B, (int)T, ndir, st);
}
