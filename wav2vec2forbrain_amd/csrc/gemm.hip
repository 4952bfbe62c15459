// LDS-tiled MFMA GEMM for gfx950 with implicit conv1d / unfold operand views and fused
// epilogues (bias, activation, dropout, activation-backward, residual).
//
// Operands live in HBM as fp32 (activations, master weights, gradients) and are converted
// while staging into LDS: bf16 for v_mfma_f32_16x16x32_bf16 (fp32 accumulate), or kept fp32
// for v_mfma_f32_16x16x4_f32 (exact-fp32 parity mode). 256 threads = 4 waves (2 x 2), each
// wave owns a (BM/2) x (BN/2) sub-tile of 16x16 MFMA tiles; K tile KB = 32 or 64; two LDS buffers with
// register staging (global loads for tile k+1 are in flight while tile k is computed).
#include "common.h"
#include "../../include/b2p_hip.h"
#include "timing.h"
#include "gemm_epi.h"
#include <stdlib.h>

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------------ operand views
struct OpState {
  const float* base;    // pointer incl. batch offset
  int64_t ld;
  // conv view
  int T_out, T_in, stride, pad, Cg;
  int64_t sample_stride;
};

__device__ __forceinline__ int64_t batch_off(const b2p_operand& o, int z1, int z2) {
  const int64_t i1 = o.gather1 ? o.gather1[z1] : (int64_t)z1;
  return i1 * o.bs1 + (int64_t)z2 * o.bs2;
}

// Precision traits -----------------------------------------------------------------
template <int PREC, int KB> struct Prec;
template <int KB> struct Prec<0, KB> {   // bf16 MFMA
  typedef __bf16 T;
  static constexpr int LDS_STRIDE = KB + 8;   // rows 16-B aligned for ds_read_b128; odd multiple of 16 B
};
template <int KB> struct Prec<1, KB> {   // fp32 MFMA
  typedef float T;
  static constexpr int LDS_STRIDE = KB + 1;
};
template <int KB> struct Prec<2, KB> {   // fp16 MFMA (same rate as bf16, 3 more mantissa bits)
  typedef _Float16 T;
  static constexpr int LDS_STRIDE = KB + 8;
};
// split bf16 ("bf16x3"): x = hi + lo with hi = bf16(x), lo = bf16(x - hi), two LDS planes; the
// product is hi*hi + hi*lo + lo*hi on bf16 MFMA (the dropped lo*lo is ~2^-18 relative): about 16
// significant bits per product at a third of the bf16 MFMA rate, five times the exact-fp32 MFMA rate
template <int KB> struct Prec<3, KB> {
  typedef __bf16 T;
  static constexpr int LDS_STRIDE = KB + 8;
};
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int PREC, int KB>
__device__ __forceinline__ void st4(typename Prec<PREC, KB>::T* dst, float a, float b, float c, float d,
                                    int plane = 0) {
  if constexpr (PREC == 3) {
    bf16x4 h = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
    bf16x4 l = {(__bf16)(a - (float)h[0]), (__bf16)(b - (float)h[1]), (__bf16)(c - (float)h[2]),
                (__bf16)(d - (float)h[3])};
    *reinterpret_cast<bf16x4*>(dst) = h;
    *reinterpret_cast<bf16x4*>(dst + plane) = l;
  } else if constexpr (PREC == 0) {
    bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
    *reinterpret_cast<bf16x4*>(dst) = v;
  } else if constexpr (PREC == 2) {
    f16x4 v = {(_Float16)b2p_f16_sat(a), (_Float16)b2p_f16_sat(b), (_Float16)b2p_f16_sat(c), (_Float16)b2p_f16_sat(d)};
    *reinterpret_cast<f16x4*>(dst) = v;
  } else {
    dst[0] = a; dst[1] = b; dst[2] = c; dst[3] = d;
  }
}

// ------------------------------------------------------------------ tile loader
// Loads an R x KB (rows = M or N index, cols = k) tile of an operand into registers and writes it
// K-contiguous into LDS: lds[row][k].
//  INNER_K: the operand's contiguous dim is k: CPR = KB/4 float4 chunks per row, RPP = NT/CPR rows
//           per pass, NV = R/RPP float4 per thread.
//  !INNER_K: contiguous dim is m/n: 4(k) x 4(mn) register blocks transposed on the way to LDS;
//           NC = R/4 mn-chunks x KG = KB/4 k-groups = NBLK blocks per thread (0.5 -> half active).
template <int R, int KB, bool INNER_K, bool CONV, int PREC>
struct Loader {
  static constexpr int CPR = KB / 4;
  static constexpr int RPP = NT / CPR;
  static constexpr int NC = R / 4, KG = KB / 4;
  static constexpr int NBLK = (NC * KG) >= NT ? (NC * KG) / NT : 1;
  static constexpr int NV = INNER_K ? R / RPP : 4 * NBLK;
  float4 v[NV];
  bool active;
  int64_t rowoff[INNER_K ? NV : 1];
  int frame0[INNER_K ? NV : 1];
  bool rowok[INNER_K ? NV : 1];
  int tap, ch;                         // INNER_K conv: k tracker; !INNER_K conv: fixed (mn) tap/ch
  int tb[INNER_K ? 1 : NBLK][4], tt[INNER_K ? 1 : NBLK][4];
  int64_t mnoff[INNER_K ? 1 : NBLK];
  int mnvalid[INNER_K ? 1 : NBLK];
  int gk[INNER_K ? 1 : NBLK];          // k-group of each block

  __device__ __forceinline__ void init(const OpState& s, int tid, int mn0, int MNdim, int kstart) {
    if constexpr (INNER_K) {
      active = true;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int row = mn0 + tid / CPR + RPP * i;
        rowok[i] = row < MNdim;
        if constexpr (CONV) {
          const int rr = rowok[i] ? row : 0;
          const int b = rr / s.T_out, t = rr - b * s.T_out;
          rowoff[i] = (int64_t)b * s.sample_stride;
          frame0[i] = t * s.stride - s.pad;
        } else {
          rowoff[i] = (int64_t)row * s.ld;
          frame0[i] = 0;
        }
      }
      const int kk = kstart + (tid % CPR) * 4;
      if constexpr (CONV) { tap = kk / s.Cg; ch = kk - tap * s.Cg; } else { tap = 0; ch = kk; }
    } else {
      active = (NC * KG >= NT) || tid < NC * KG;
#pragma unroll
      for (int q = 0; q < NBLK; ++q) {
        const int bidx = tid + NT * q;
        const int c = bidx % NC, g = bidx / NC;
        gk[q] = g;
        const int mn = mn0 + 4 * c;
        mnvalid[q] = MNdim - mn;
        if constexpr (CONV) {
          const int mm = mnvalid[q] > 0 ? mn : 0;
          const int tp = mm / s.Cg, cc = mm - tp * s.Cg;
          mnoff[q] = (int64_t)(tp - s.pad) * s.ld + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int k = kstart + 4 * g + j;
            tb[q][j] = k / s.T_out; tt[q][j] = k - tb[q][j] * s.T_out;
          }
          tbtap[q] = tp;   // frame = tt*stride + tap - pad (validity), address via mnoff
        } else {
          mnoff[q] = mn;
        }
      }
    }
  }
  int tbtap[INNER_K ? 1 : NBLK];

  __device__ __forceinline__ static float4 sel4(float4 x, bool ok, int nvalid) {
    x.x = ok ? x.x : 0.f;
    x.y = (ok && nvalid > 1) ? x.y : 0.f;
    x.z = (ok && nvalid > 2) ? x.z : 0.f;
    x.w = (ok && nvalid > 3) ? x.w : 0.f;
    return x;
  }

  // Branch-free loads: every lane issues one unconditional 16-B load (from a clamped, always
  // in-bounds address when the element is outside the operand) and zeroes invalid elements with
  // selects, so the global loads of a K-step stay in flight together (a per-load branch makes
  // hipcc wait vmcnt(0) per load). In-bounds guarantee: ld % 4 == 0 => ld >= roundup4(dim).
  __device__ __forceinline__ void load(const OpState& s, int tid, int k0, int Kdim) {
    if constexpr (INNER_K) {
      const int kk = k0 + (tid % CPR) * 4;
      const int kvalid = Kdim - kk;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        bool ok = rowok[i] && kvalid > 0;
        const float* p;
        if constexpr (CONV) {
          const int f = frame0[i] + tap;
          ok = ok && f >= 0 && f < s.T_in;
          p = ok ? s.base + rowoff[i] + (int64_t)f * s.ld + ch : s.base;
        } else {
          p = ok ? s.base + rowoff[i] + kk : s.base;
        }
        v[i] = sel4(*reinterpret_cast<const float4*>(p), ok, kvalid);
      }
      if constexpr (CONV) {
        ch += KB;
        while (ch >= s.Cg) { ch -= s.Cg; ++tap; }
      }
    } else {
      if (!active) return;
#pragma unroll
      for (int q = 0; q < NBLK; ++q) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + 4 * gk[q] + j;
          bool ok = k < Kdim && mnvalid[q] > 0;
          const float* p;
          if constexpr (CONV) {
            const int f = tt[q][j] * s.stride + tbtap[q] - s.pad;
            ok = ok && f >= 0 && f < s.T_in;
            p = ok ? s.base + (int64_t)tb[q][j] * s.sample_stride + (int64_t)(tt[q][j] * s.stride) * s.ld + mnoff[q]
                   : s.base;
            tt[q][j] += KB;
            while (tt[q][j] >= s.T_out) { tt[q][j] -= s.T_out; ++tb[q][j]; }
          } else {
            p = ok ? s.base + (int64_t)k * s.ld + mnoff[q] : s.base;
          }
          v[4 * q + j] = sel4(*reinterpret_cast<const float4*>(p), ok, mnvalid[q]);
        }
      }
    }
  }

  __device__ __forceinline__ void store(typename Prec<PREC, KB>::T* lds, int tid, int plane = 0) {
    constexpr int LS = Prec<PREC, KB>::LDS_STRIDE;
    if constexpr (INNER_K) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int row = tid / CPR + RPP * i;
        st4<PREC, KB>(lds + row * LS + (tid % CPR) * 4, v[i].x, v[i].y, v[i].z, v[i].w, plane);
      }
    } else {
      if (!active) return;
#pragma unroll
      for (int q = 0; q < NBLK; ++q) {
        const int bidx = tid + NT * q;
        const int c = bidx % NC, g = bidx / NC;
        typename Prec<PREC, KB>::T* d = lds + (4 * c) * LS + 4 * g;
        const float4* w = v + 4 * q;
        st4<PREC, KB>(d + 0 * LS, w[0].x, w[1].x, w[2].x, w[3].x, plane);
        st4<PREC, KB>(d + 1 * LS, w[0].y, w[1].y, w[2].y, w[3].y, plane);
        st4<PREC, KB>(d + 2 * LS, w[0].z, w[1].z, w[2].z, w[3].z, plane);
        st4<PREC, KB>(d + 3 * LS, w[0].w, w[1].w, w[2].w, w[3].w, plane);
      }
    }
  }
};

__device__ __forceinline__ OpState make_state(const b2p_operand& o, int z1, int z2) {
  OpState s;
  s.base = static_cast<const float*>(o.ptr) + batch_off(o, z1, z2);
  s.ld = o.ld;
  s.T_out = o.conv_T_out > 0 ? o.conv_T_out : 1;
  s.T_in = o.conv_T_in;
  s.stride = o.conv_stride;
  s.pad = o.conv_pad;
  s.Cg = o.conv_Cg > 0 ? o.conv_Cg : 1;
  s.sample_stride = o.conv_sample_stride;
  return s;
}

// ------------------------------------------------------------------ kernel
template <int BM, int BN, int KB, bool AK, bool BKin, bool ACONV, bool BCONV, int PREC>
__global__ void __launch_bounds__(NT) gemm_kernel(const b2p_gemm_desc d, const EpiArgs ea) {
  typedef typename Prec<PREC, KB>::T T;
  constexpr int LS = Prec<PREC, KB>::LDS_STRIDE;
  constexpr int WM = BM / 2, WN = BN / 2;     // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;   // 16x16 MFMA tiles per wave
  // split bf16: the lo plane follows the two hi buffers
  constexpr int PLANE = PREC == 3 ? 2 * (BM + BN) * LS : 0;
  __shared__ __attribute__((aligned(16))) T smem[(PREC == 3 ? 2 : 1) * 2 * (BM + BN) * LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // blockIdx.z = batch index * ksplit + K-slice index
  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  const int z = blockIdx.z / ks, ksl = blockIdx.z - (blockIdx.z / ks) * ks;
  const int z1 = z / d.nz2, z2 = z - z1 * d.nz2;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = (int)d.M, N = (int)d.N;
  const int kchunk = ks > 1 ? (int)d.kchunk : (int)d.K;   // multiple of KB
  const int kbeg = ksl * kchunk;
  const int K = ((int)d.K < kbeg + kchunk) ? (int)d.K : kbeg + kchunk;   // exclusive end

  OpState sa = make_state(d.A, z1, z2);
  OpState sb = make_state(d.B, z1, z2);
  Loader<BM, KB, AK, ACONV, PREC> la;
  Loader<BN, KB, BKin, BCONV, PREC> lb;
  la.init(sa, tid, m0, M, kbeg);
  lb.init(sb, tid, n0, N, kbeg);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // buffer b: A at smem + b*(BM+BN)*LS, B right after it
#define AS_(b) (smem + (b) * (BM + BN) * LS)
#define BS_(b) (smem + (b) * (BM + BN) * LS + BM * LS)

  const int nk = (K > kbeg && !b2p_gated_off(ea.gate)) ? (K - kbeg + KB - 1) / KB : 0;
  la.load(sa, tid, kbeg, K);
  lb.load(sb, tid, kbeg, K);
  la.store(AS_(0), tid, PLANE);
  lb.store(BS_(0), tid, PLANE);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(sa, tid, kbeg + (kt + 1) * KB, K);
      lb.load(sb, tid, kbeg + (kt + 1) * KB, K);
    }
    const T* A_ = AS_(cur);
    const T* B_ = BS_(cur);
    if constexpr (PREC == 0) {
#pragma unroll
      for (int kk = 0; kk < KB / 32; ++kk) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(A_ + (wm * WM + i * 16 + (lane & 15)) * LS + 32 * kk + 8 * (lane >> 4));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(B_ + (wn * WN + j * 16 + (lane & 15)) * LS + 32 * kk + 8 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else if constexpr (PREC == 3) {
#pragma unroll
      for (int kk = 0; kk < KB / 32; ++kk) {
        bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int o = (wm * WM + i * 16 + (lane & 15)) * LS + 32 * kk + 8 * (lane >> 4);
          ah[i] = *reinterpret_cast<const bf16x8*>(A_ + o);
          al[i] = *reinterpret_cast<const bf16x8*>(A_ + PLANE + o);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int o = (wn * WN + j * 16 + (lane & 15)) * LS + 32 * kk + 8 * (lane >> 4);
          bh[j] = *reinterpret_cast<const bf16x8*>(B_ + o);
          bl[j] = *reinterpret_cast<const bf16x8*>(B_ + PLANE + o);
        }
        // the two correction products first, then the leading one
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (PREC == 2) {
#pragma unroll
      for (int kk = 0; kk < KB / 32; ++kk) {
        f16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const f16x8*>(A_ + (wm * WM + i * 16 + (lane & 15)) * LS + 32 * kk + 8 * (lane >> 4));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const f16x8*>(B_ + (wn * WN + j * 16 + (lane & 15)) * LS + 32 * kk + 8 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KB / 4; ++ks) {
        float af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = A_[(wm * WM + i * 16 + (lane & 15)) * LS + 4 * ks + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = B_[(wn * WN + j * 16 + (lane & 15)) * LS + 4 * ks + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      la.store(AS_(cur ^ 1), tid, PLANE);
      lb.store(BS_(cur ^ 1), tid, PLANE);
    }
    __syncthreads();
  }

  // epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each 16x16 tile. The split-K
  // branch is hoisted out of the unrolled loops so acc[][] keeps constant indices (registers).
  if (ks > 1) {
    float* slab = d.workspace + ((int64_t)z * ks + ksl) * (int64_t)M * N;
#pragma clang loop unroll(full)
    for (int i = 0; i < TM; ++i)
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j)
#pragma clang loop unroll(full)
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WN + j * 16 + (lane & 15);
          if (m < M && n < N) slab[(int64_t)m * N + n] = acc[i][j][r];
        }
  } else {
#pragma clang loop unroll(full)
    for (int i = 0; i < TM; ++i)
#pragma clang loop unroll(full)
      for (int j = 0; j < TN; ++j)
#pragma clang loop unroll(full)
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WN + j * 16 + (lane & 15);
          epilogue_store(ea, z, z1, z2, m, n, acc[i][j][r]);
        }
  }
#undef AS_
#undef BS_
}

// K-tile selection: B2P_GEMM_KB=32|64 (default 64 for bf16; fp32 parity mode keeps 32 so its
// LDS footprint stays at 2 x (BM+BN) x 33 floats).
int kb_choice() {
  static int kb = [] {
    const char* e = getenv("B2P_GEMM_KB");
    const int v = e ? atoi(e) : 64;
    return v == 32 ? 32 : 64;
  }();
  return kb;
}

template <int BM, int BN, bool AK, bool BKin, bool ACONV, bool BCONV>
int launch_prec(const b2p_gemm_desc& d, const EpiArgs& ea, hipStream_t st) {
  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  dim3 grid((unsigned)((d.N + BN - 1) / BN), (unsigned)((d.M + BM - 1) / BM), (unsigned)(d.nz1 * d.nz2 * ks));
  if (d.precision == 1)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 32, AK, BKin, ACONV, BCONV, 1>), grid, dim3(NT), 0, st, d, ea);
  else if (d.precision == 3)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 32, AK, BKin, ACONV, BCONV, 3>), grid, dim3(NT), 0, st, d, ea);
  else if (d.precision == 2 && (ks == 1 || d.kchunk % 64 == 0))
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 64, AK, BKin, ACONV, BCONV, 2>), grid, dim3(NT), 0, st, d, ea);
  else if (d.precision == 2)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 32, AK, BKin, ACONV, BCONV, 2>), grid, dim3(NT), 0, st, d, ea);
  else if (kb_choice() == 64 && (ks == 1 || d.kchunk % 64 == 0))
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 64, AK, BKin, ACONV, BCONV, 0>), grid, dim3(NT), 0, st, d, ea);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 32, AK, BKin, ACONV, BCONV, 0>), grid, dim3(NT), 0, st, d, ea);
  return 0;
}

template <bool AK, bool BKin, bool ACONV, bool BCONV>
int launch_tiles(const b2p_gemm_desc& d, const EpiArgs& ea, hipStream_t st) {
  // narrow-N problems (pos-conv groups N=48, lm_head N=32) use a 128x64 tile
  if (d.N <= 64) return launch_prec<128, 64, AK, BKin, ACONV, BCONV>(d, ea, st);
  return launch_prec<128, 128, AK, BKin, ACONV, BCONV>(d, ea, st);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_operand(const b2p_operand& o, const char* name) {
  B2P_CHECK_ARG(o.ptr != nullptr, "gemm: operand %s is NULL", name);
  B2P_CHECK_ARG(aligned16(o.ptr), "gemm: operand %s not 16-byte aligned", name);
  B2P_CHECK_ARG(o.dtype >= 0 && o.dtype <= 2, "gemm: operand %s dtype must be 0 (fp32), 1 (bf16) or 2 (fp16)", name);
  const int64_t v = o.dtype != 0 ? 8 : 4;   // elements per 16-byte vector
  B2P_CHECK_ARG(o.ld % v == 0 && o.bs1 % v == 0 && o.bs2 % v == 0,
                "gemm: operand %s strides must be multiples of %lld (ld=%lld)", name, (long long)v, (long long)o.ld);
  if (o.conv) {
    B2P_CHECK_ARG(o.conv_Cg > 0 && o.conv_Cg % v == 0, "gemm: operand %s conv_Cg must be a multiple of %lld", name,
                  (long long)v);
    B2P_CHECK_ARG(o.conv_sample_stride % v == 0, "gemm: operand %s conv sample stride %% %lld", name, (long long)v);
    B2P_CHECK_ARG(o.conv_T_out > 0 && o.conv_T_in > 0 && o.conv_stride > 0, "gemm: operand %s bad conv geometry", name);
  }
  return 0;
}

}  // namespace

extern "C" int b2p_gemm(const b2p_gemm_desc* dp, b2p_stream_t stream) {
  B2P_CHECK_ARG(dp != nullptr, "gemm: NULL descriptor");
  const b2p_gemm_desc& d = *dp;
  B2P_CHECK_ARG(d.M >= 0 && d.N >= 0 && d.K >= 0, "gemm: negative size");
  B2P_CHECK_ARG(d.M < (1ll << 31) && d.N < (1ll << 31) && d.K < (1ll << 31), "gemm: size too large");
  B2P_CHECK_ARG(d.nz1 >= 1 && d.nz2 >= 1, "gemm: batch dims must be >= 1");
  B2P_CHECK_ARG(d.precision >= 0 && d.precision <= 3,
                "gemm: precision must be 0 (bf16), 1 (fp32), 2 (fp16) or 3 (split bf16)");
  if (d.M == 0 || d.N == 0) return 0;
  B2P_CHECK_ARG(d.ep.C != nullptr || d.ep.C16 != nullptr, "gemm: C and C16 are NULL");
  B2P_CHECK_ARG(d.ep.C != nullptr || d.ep.beta == 0.f, "gemm: beta != 0 needs C");
  if (check_operand(d.A, "A") || check_operand(d.B, "B")) return 1;
  B2P_CHECK_ARG(d.A.dtype == d.B.dtype, "gemm: operands must share a dtype");
  const bool bf16_ops = d.A.dtype != 0;   // 16-bit operands: the LDS-DMA kernel (gemm16.hip)
  B2P_CHECK_ARG(!b2p_gate_batch() || bf16_ops, "gemm: per-member gates (b2p_set_gate_batch) need 16-bit operands");
  if (bf16_ops) {
    B2P_CHECK_ARG(d.precision == (d.A.dtype == 1 ? 0 : 2), "gemm: bf16 operands need precision 0, fp16 precision 2");
    B2P_CHECK_ARG(!(d.A.inner_is_k || d.B.inner_is_k) || d.K % 8 == 0,
                  "gemm: bf16 k-contiguous operand needs K %% 8 == 0 (K=%lld)", (long long)d.K);
    B2P_CHECK_ARG(!d.B.conv, "gemm: bf16 path supports a conv view on A only");
    B2P_CHECK_ARG(!d.A.conv || d.A.inner_is_k, "gemm: bf16 conv view needs A inner=k");
  }
  B2P_CHECK_ARG(!(d.A.conv && d.B.conv), "gemm: at most one implicit-conv operand");
  if (d.ep.act_bwd != B2P_ACT_NONE) B2P_CHECK_ARG(d.ep.aux != nullptr || d.ep.aux16 != nullptr, "gemm: act_bwd needs aux");
  if (d.ep.pre16 || d.ep.aux16 || d.ep.colsum_part || d.ep.C16b) {
    B2P_CHECK_ARG(bf16_ops, "gemm: pre16 / aux16 / colsum_part / C16b need the bf16-operand kernel");
    B2P_CHECK_ARG(!d.ep.C16b || d.ksplit <= 1, "gemm: C16b needs a launch without split-K");
    B2P_CHECK_ARG(!d.ep.colsum_part || (d.nz1 * d.nz2 == 1 && d.ksplit <= 1 && d.N % 4 == 0),
                  "gemm: colsum_part needs nz1*nz2 == 1, no split-K and N %% 4 == 0");
  }
  B2P_CHECK_ARG(d.ep.drop_p >= 0.f && d.ep.drop_p < 1.f, "gemm: dropout p must be in [0,1)");
  if (d.ksplit > 1) {
    B2P_CHECK_ARG(d.workspace != nullptr, "gemm: split-K needs a workspace");
    B2P_CHECK_ARG(d.kchunk > 0 && d.kchunk % (bf16_ops ? 64 : 32) == 0 && (int64_t)d.kchunk * d.ksplit >= d.K,
                  "gemm: kchunk must be a multiple of %d covering K", bf16_ops ? 64 : 32);
    B2P_CHECK_ARG(d.workspace_floats >= (int64_t)d.ksplit * d.nz1 * d.nz2 * d.M * d.N, "gemm: split-K workspace too small");
    B2P_CHECK_ARG(!d.ep.bias && !d.ep.pre_out && d.ep.act == 0 && d.ep.act_bwd == 0 && d.ep.drop_p == 0.f &&
                  !d.ep.residual, "gemm: split-K supports alpha/beta epilogues only");
  }

  const EpiArgs ea = make_epi_args(d);

  hipStream_t st = (hipStream_t)stream;
  b2p_timing_begin(d.timing_family, st);
  const bool AK = d.A.inner_is_k != 0, BKn = d.B.inner_is_k != 0;
  int rc;
  if (bf16_ops) {
    B2P_CHECK_ARG(AK || !BKn, "gemm: A inner=m with B inner=k layout not supported");
    rc = b2p_gemm16_launch(d, st);
  } else if (AK && BKn) {
    if (d.A.conv) rc = launch_tiles<true, true, true, false>(d, ea, st);
    else if (d.B.conv) { b2p_set_error("gemm: conv view on B requires B inner=n"); return 1; }
    else rc = launch_tiles<true, true, false, false>(d, ea, st);
  } else if (AK && !BKn) {
    B2P_CHECK_ARG(!d.A.conv && !d.B.conv, "gemm: NN layout does not support conv views");
    rc = launch_tiles<true, false, false, false>(d, ea, st);
  } else if (!AK && !BKn) {
    B2P_CHECK_ARG(!d.A.conv, "gemm: TN layout supports a conv view on B only");
    if (d.B.conv) rc = launch_tiles<false, false, false, true>(d, ea, st);
    else rc = launch_tiles<false, false, false, false>(d, ea, st);
  } else {
    b2p_set_error("gemm: A inner=m with B inner=k layout not supported");
    return 1;
  }
  if (rc) return rc;
  if (d.ksplit > 1 && !(bf16_ops && gemm16_splitk_fused(d))) {
    const int64_t total = (int64_t)d.nz1 * d.nz2 * d.M * d.N;
    const b2p_epilogue& e = d.ep;
    const bool v4 = d.N % 4 == 0 && e.ldc % 4 == 0 && e.cbs1 % 4 == 0 && e.cbs2 % 4 == 0 &&
                    ((uintptr_t)e.C & 15u) == 0 && ((uintptr_t)e.C16 & 7u) == 0 && ((uintptr_t)d.workspace & 15u) == 0;
    if (v4)
      hipLaunchKernelGGL(splitk_reduce4, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0, st, d.workspace,
                         d.ksplit, d.M, d.N, d.nz2, d.ep, total / 4);
    else
      hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, d.workspace,
                         d.ksplit, d.M, d.N, d.nz2, d.ep, total);
  }
  B2P_CHECK_LAUNCH();
  b2p_timing_end(d.timing_family, st, d.flops);
  return 0;
}
