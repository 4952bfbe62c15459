// LDS-tiled MFMA GEMM for gfx950 with implicit conv1d / unfold operand views and fused
// epilogues (bias, activation, dropout, activation-backward, residual).
//
// Operands live in HBM as fp32 (activations, master weights, gradients) and are converted
// while staging into LDS: bf16 for v_mfma_f32_16x16x32_bf16 (fp32 accumulate), or kept fp32
// for v_mfma_f32_16x16x4_f32 (exact-fp32 parity mode). 256 threads = 4 waves (2 x 2), each
// wave owns a (BM/2) x (BN/2) sub-tile of 16x16 MFMA tiles; BK = 32; two LDS buffers with
// register staging (global loads for tile k+1 are in flight while tile k is computed).
#include "common.h"
#include "../../include/b2p_hip.h"
#include "timing.h"

namespace {

constexpr int BK = 32;
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
template <int PREC> struct Prec;
template <> struct Prec<0> {   // bf16 MFMA
  typedef __bf16 T;
  static constexpr int LDS_STRIDE = BK + 8;   // 80 B rows: 16-B aligned ds_read_b128
};
template <> struct Prec<1> {   // fp32 MFMA
  typedef float T;
  static constexpr int LDS_STRIDE = BK + 1;
};

template <int PREC>
__device__ __forceinline__ void st4(typename Prec<PREC>::T* dst, float a, float b, float c, float d) {
  if constexpr (PREC == 0) {
    bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
    *reinterpret_cast<bf16x4*>(dst) = v;
  } else {
    dst[0] = a; dst[1] = b; dst[2] = c; dst[3] = d;
  }
}

// ------------------------------------------------------------------ tile loader
// Loads an R x BK (rows = M or N index, cols = k) tile of an operand into registers and
// writes it K-contiguous into LDS: lds[row][k].
template <int R, bool INNER_K, bool CONV, int PREC>
struct Loader {
  static constexpr int NV = INNER_K ? R / 32 : 4;  // float4 registers per thread
  float4 v[NV];
  bool active;
  // INNER_K: per-row precomputed frame / row offsets, one k-tracker
  int64_t rowoff[INNER_K ? R / 32 : 1];
  int frame0[INNER_K ? R / 32 : 1];
  bool rowok[INNER_K ? R / 32 : 1];
  int tap, ch;          // conv tracker for inner index (INNER_K: k; !INNER_K: mn fixed)
  // !INNER_K: per-k-row trackers
  int tb[4], tt[4];
  int64_t mnoff;        // !INNER_K: fixed inner offset (mn) part
  int mnvalid;          // number of valid inner elements at this thread's chunk

  __device__ __forceinline__ void init(const OpState& s, int tid, int mn0, int MNdim, int kstart) {
    if constexpr (INNER_K) {
      active = true;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int row = mn0 + (tid >> 3) + 32 * i;
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
      const int kk = kstart + (tid & 7) * 4;
      if constexpr (CONV) { tap = kk / s.Cg; ch = kk - tap * s.Cg; } else { tap = 0; ch = kk; }
    } else {
      // R/4 mn-chunks x 8 k-groups of 4
      const int nchunk = R / 4;
      const int c = tid % nchunk, g = tid / nchunk;
      active = g < 8;
      const int mn = mn0 + 4 * c;
      mnvalid = MNdim - mn;
      if constexpr (CONV) {
        const int mm = mnvalid > 0 ? mn : 0;
        tap = mm / s.Cg; ch = mm - tap * s.Cg;
        mnoff = (int64_t)(tap - s.pad) * s.ld + ch;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = kstart + 4 * g + j;   // first k-tile of this block's K range
          tb[j] = k / s.T_out; tt[j] = k - tb[j] * s.T_out;
        }
      } else {
        mnoff = mn;
      }
    }
  }

  // Branch-free loads: every lane issues one unconditional 16-B load (from a clamped, always
  // in-bounds address when the element is outside the operand) and zeroes invalid elements with
  // selects, so the global loads of a K-step stay in flight together (a per-load branch makes
  // hipcc wait vmcnt(0) per load). In-bounds guarantee: ld % 4 == 0 => ld >= roundup4(dim).
  __device__ __forceinline__ static float4 sel4(float4 x, bool ok, int nvalid) {
    x.x = ok ? x.x : 0.f;
    x.y = (ok && nvalid > 1) ? x.y : 0.f;
    x.z = (ok && nvalid > 2) ? x.z : 0.f;
    x.w = (ok && nvalid > 3) ? x.w : 0.f;
    return x;
  }

  __device__ __forceinline__ void load(const OpState& s, int tid, int k0, int Kdim) {
    if constexpr (INNER_K) {
      const int kk = k0 + (tid & 7) * 4;
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
        ch += BK;
        while (ch >= s.Cg) { ch -= s.Cg; ++tap; }
      }
    } else {
      if (!active) return;
      const int nchunk = R / 4;
      const int g = tid / nchunk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 4 * g + j;
        bool ok = k < Kdim && mnvalid > 0;
        const float* p;
        if constexpr (CONV) {
          const int f = tt[j] * s.stride + tap - s.pad;
          ok = ok && f >= 0 && f < s.T_in;
          p = ok ? s.base + (int64_t)tb[j] * s.sample_stride + (int64_t)(tt[j] * s.stride) * s.ld + mnoff : s.base;
          tt[j] += BK;
          while (tt[j] >= s.T_out) { tt[j] -= s.T_out; ++tb[j]; }
        } else {
          p = ok ? s.base + (int64_t)k * s.ld + mnoff : s.base;
        }
        v[j] = sel4(*reinterpret_cast<const float4*>(p), ok, mnvalid);
      }
    }
  }

  __device__ __forceinline__ void store(typename Prec<PREC>::T* lds, int tid) {
    constexpr int LS = Prec<PREC>::LDS_STRIDE;
    if constexpr (INNER_K) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int row = (tid >> 3) + 32 * i;
        st4<PREC>(lds + row * LS + (tid & 7) * 4, v[i].x, v[i].y, v[i].z, v[i].w);
      }
    } else {
      if (!active) return;
      const int nchunk = R / 4;
      const int c = tid % nchunk, g = tid / nchunk;
      typename Prec<PREC>::T* d = lds + (4 * c) * LS + 4 * g;
      st4<PREC>(d + 0 * LS, v[0].x, v[1].x, v[2].x, v[3].x);
      st4<PREC>(d + 1 * LS, v[0].y, v[1].y, v[2].y, v[3].y);
      st4<PREC>(d + 2 * LS, v[0].z, v[1].z, v[2].z, v[3].z);
      st4<PREC>(d + 3 * LS, v[0].w, v[1].w, v[2].w, v[3].w);
    }
  }
};

__device__ __forceinline__ OpState make_state(const b2p_operand& o, int z1, int z2) {
  OpState s;
  s.base = o.ptr + batch_off(o, z1, z2);
  s.ld = o.ld;
  s.T_out = o.conv_T_out > 0 ? o.conv_T_out : 1;
  s.T_in = o.conv_T_in;
  s.stride = o.conv_stride;
  s.pad = o.conv_pad;
  s.Cg = o.conv_Cg > 0 ? o.conv_Cg : 1;
  s.sample_stride = o.conv_sample_stride;
  return s;
}

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
  v = apply_act(v, e.act);
  if (e.drop_p > 0.0f) {
    const uint64_t idx = ((uint64_t)z * (uint64_t)a.M + (uint64_t)m) * (uint64_t)a.N + (uint64_t)n;
    v = b2p_keep(e.drop_seed, idx, a.drop_thr) ? v * a.drop_scale : 0.0f;
  }
  if (e.act_bwd != B2P_ACT_NONE) {
    const float x = e.aux[(int64_t)z1 * e.abs1 + (int64_t)z2 * e.abs2 + (int64_t)m * e.ldaux + n];
    v *= act_grad(x, e.act_bwd);
  }
  if (e.residual) v += e.residual[(int64_t)z1 * e.rbs1 + (int64_t)z2 * e.rbs2 + (int64_t)m * e.ldr + n];
  e.C[coff] = v;
}

// ------------------------------------------------------------------ kernel
template <int BM, int BN, bool AK, bool BKin, bool ACONV, bool BCONV, int PREC>
__global__ void __launch_bounds__(NT) gemm_kernel(const b2p_gemm_desc d, const EpiArgs ea) {
  typedef typename Prec<PREC>::T T;
  constexpr int LS = Prec<PREC>::LDS_STRIDE;
  constexpr int WM = BM / 2, WN = BN / 2;     // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;   // 16x16 MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) T smem[2 * (BM + BN) * LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // blockIdx.z = batch index * ksplit + K-slice index
  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  const int z = blockIdx.z / ks, ksl = blockIdx.z - (blockIdx.z / ks) * ks;
  const int z1 = z / d.nz2, z2 = z - z1 * d.nz2;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = (int)d.M, N = (int)d.N;
  const int kchunk = ks > 1 ? (int)d.kchunk : (int)d.K;   // multiple of BK
  const int kbeg = ksl * kchunk;
  const int K = ((int)d.K < kbeg + kchunk) ? (int)d.K : kbeg + kchunk;   // exclusive end

  OpState sa = make_state(d.A, z1, z2);
  OpState sb = make_state(d.B, z1, z2);
  Loader<BM, AK, ACONV, PREC> la;
  Loader<BN, BKin, BCONV, PREC> lb;
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

  const int nk = K > kbeg ? (K - kbeg + BK - 1) / BK : 0;
  la.load(sa, tid, kbeg, K);
  lb.load(sb, tid, kbeg, K);
  la.store(AS_(0), tid);
  lb.store(BS_(0), tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(sa, tid, kbeg + (kt + 1) * BK, K);
      lb.load(sb, tid, kbeg + (kt + 1) * BK, K);
    }
    const T* A_ = AS_(cur);
    const T* B_ = BS_(cur);
    if constexpr (PREC == 0) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A_ + (wm * WM + i * 16 + (lane & 15)) * LS + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(B_ + (wn * WN + j * 16 + (lane & 15)) * LS + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
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
      la.store(AS_(cur ^ 1), tid);
      lb.store(BS_(cur ^ 1), tid);
    }
    __syncthreads();
  }

  // epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each 16x16 tile. The split-K
  // branch is hoisted out of the unrolled loops so acc[][] keeps constant indices (registers).
  if (ks > 1) {
    float* slab = d.workspace + ((int64_t)z * ks + ksl) * (int64_t)M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WN + j * 16 + (lane & 15);
          if (m < M && n < N) slab[(int64_t)m * N + n] = acc[i][j][r];
        }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const int n = n0 + wn * WN + j * 16 + (lane & 15);
          epilogue_store(ea, z, z1, z2, m, n, acc[i][j][r]);
        }
  }
#undef AS_
#undef BS_
}

template <int BM, int BN, bool AK, bool BKin, bool ACONV, bool BCONV>
int launch_prec(const b2p_gemm_desc& d, const EpiArgs& ea, hipStream_t st) {
  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  dim3 grid((unsigned)((d.N + BN - 1) / BN), (unsigned)((d.M + BM - 1) / BM), (unsigned)(d.nz1 * d.nz2 * ks));
  if (d.precision == 1)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BKin, ACONV, BCONV, 1>), grid, dim3(NT), 0, st, d, ea);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BKin, ACONV, BCONV, 0>), grid, dim3(NT), 0, st, d, ea);
  return 0;
}

template <bool AK, bool BKin, bool ACONV, bool BCONV>
int launch_tiles(const b2p_gemm_desc& d, const EpiArgs& ea, hipStream_t st) {
  // narrow-N problems (pos-conv groups N=48, lm_head N=32) use a 128x64 tile
  if (d.N <= 64) return launch_prec<128, 64, AK, BKin, ACONV, BCONV>(d, ea, st);
  return launch_prec<128, 128, AK, BKin, ACONV, BCONV>(d, ea, st);
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
  float* c = e.C + z1 * e.cbs1 + z2 * e.cbs2 + m * e.ldc + n;
  float v = e.alpha * s;
  if (e.beta != 0.f) v += e.beta * *c;
  *c = v;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_operand(const b2p_operand& o, const char* name) {
  B2P_CHECK_ARG(o.ptr != nullptr, "gemm: operand %s is NULL", name);
  B2P_CHECK_ARG(aligned16(o.ptr), "gemm: operand %s not 16-byte aligned", name);
  B2P_CHECK_ARG(o.ld % 4 == 0 && o.bs1 % 4 == 0 && o.bs2 % 4 == 0,
                "gemm: operand %s strides must be multiples of 4 (ld=%lld)", name, (long long)o.ld);
  if (o.conv) {
    B2P_CHECK_ARG(o.conv_Cg > 0 && o.conv_Cg % 4 == 0, "gemm: operand %s conv_Cg must be a multiple of 4", name);
    B2P_CHECK_ARG(o.conv_sample_stride % 4 == 0, "gemm: operand %s conv sample stride %% 4", name);
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
  B2P_CHECK_ARG(d.precision == 0 || d.precision == 1, "gemm: precision must be 0 or 1");
  if (d.M == 0 || d.N == 0) return 0;
  B2P_CHECK_ARG(d.ep.C != nullptr, "gemm: C is NULL");
  if (check_operand(d.A, "A") || check_operand(d.B, "B")) return 1;
  B2P_CHECK_ARG(!(d.A.conv && d.B.conv), "gemm: at most one implicit-conv operand");
  if (d.ep.act_bwd != B2P_ACT_NONE) B2P_CHECK_ARG(d.ep.aux != nullptr, "gemm: act_bwd needs aux");
  B2P_CHECK_ARG(d.ep.drop_p >= 0.f && d.ep.drop_p < 1.f, "gemm: dropout p must be in [0,1)");
  if (d.ksplit > 1) {
    B2P_CHECK_ARG(d.workspace != nullptr, "gemm: split-K needs a workspace");
    B2P_CHECK_ARG(d.kchunk > 0 && d.kchunk % 32 == 0 && (int64_t)d.kchunk * d.ksplit >= d.K,
                  "gemm: kchunk must be a multiple of 32 covering K");
    B2P_CHECK_ARG(d.workspace_floats >= (int64_t)d.ksplit * d.nz1 * d.nz2 * d.M * d.N, "gemm: split-K workspace too small");
    B2P_CHECK_ARG(!d.ep.bias && !d.ep.pre_out && d.ep.act == 0 && d.ep.act_bwd == 0 && d.ep.drop_p == 0.f &&
                  !d.ep.residual, "gemm: split-K supports alpha/beta epilogues only");
  }

  EpiArgs ea;
  ea.e = d.ep;
  ea.M = d.M;
  ea.N = d.N;
  ea.drop_thr = b2p_dropout_threshold(d.ep.drop_p);
  ea.drop_scale = d.ep.drop_p > 0.f ? 1.0f / (1.0f - d.ep.drop_p) : 1.0f;

  hipStream_t st = (hipStream_t)stream;
  b2p_timing_begin(d.timing_family, st);
  const bool AK = d.A.inner_is_k != 0, BKn = d.B.inner_is_k != 0;
  int rc;
  if (AK && BKn) {
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
  if (d.ksplit > 1) {
    const int64_t total = (int64_t)d.nz1 * d.nz2 * d.M * d.N;
    hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, d.workspace,
                       d.ksplit, d.M, d.N, d.nz2, d.ep, total);
  }
  B2P_CHECK_LAUNCH();
  b2p_timing_end(d.timing_family, st, d.flops);
  return 0;
}
