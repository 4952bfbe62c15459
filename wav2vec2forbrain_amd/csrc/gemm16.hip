// bf16-operand GEMM for gfx950: operands live in HBM as bf16 and are copied straight into LDS
// with global_load_lds_dwordx4 (no VGPR staging, no conversion), then fed to
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
//
// Tile 128 x 128 x KT (KT = 64 or 32), 256 threads = 4 waves (2 x 2), each wave a 64 x 64 sub-tile
// (4 x 4 MFMA tiles); S LDS stages with S-1 tiles in flight behind counted vmcnt waits and raw
// s_barrier (a __syncthreads() would drain every outstanding DMA); the epilogue is staged through
// LDS so C / bias / aux / residual move as 16-byte vectors.
//
// LDS images (byte offsets inside one 16 KB operand stage; every glds wave-instruction writes
// 1024 contiguous bytes, lane L at +16*L, so swizzles are applied to the GLOBAL source address):
//  * k-contiguous operand ([row][KT k]): chunk c (8 k-values) of row r is stored in slot
//    c ^ swz_k(r). A ds_read_b128 fragment read (16 rows x one chunk per 16-lane group) then
//    covers all 64 banks once: conflict-free (measured SQ_LDS_BANK_CONFLICT = 0).
//  * m/n-contiguous operand ([64 k][128 mn], 256-B rows): chunk c of row r in slot
//    c ^ (((r & 3) << 2) | ((r >> 2) & 3)); read with ds_read_b64_tr_b16 (4 k-rows x 16 columns per
//    16-lane group, delivered column-major = the MFMA operand layout).
//
// Elements outside the operand (k >= K, rows >= M/N, conv frames outside [0, T_in)) are loaded
// from a 16-byte zero page instead, so the loads stay branch-free.
#include "common.h"
#include "../../include/b2p_hip.h"
#include "gemm_epi.h"
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

namespace {

constexpr int NT16 = 256;
constexpr int TILE = 128;

__device__ __attribute__((aligned(16))) uint32_t g_zero_page[8];   // zero-initialised

typedef __attribute__((address_space(3))) void lds_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8g __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void glds16(const void* src, lds_t* dst) {
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// swizzle of a k-contiguous image with 2*KT-byte rows (slot = chunk ^ swz_k(row)); both make a
// 16x32 ds_read_b128 fragment read conflict-free (each 16-lane group covers all 64 banks once)
template <int KT>
__device__ __forceinline__ int swz_k(int r) {
  if constexpr (KT == 64) return (r >> 1) & 7;
  else return ((r >> 3) & 1) << 1;
}
// swizzle of an mn-contiguous image with 256-B rows (128 bf16), for ds_read_b64_tr_b16
__device__ __forceinline__ int swz_t(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// per-lane source state of one ROWS x KT operand tile (NWAVES waves issue it together)
template <int ROWS, int KT, bool INNER_K, bool CONV, int NWAVES>
struct Src {
  static constexpr int NJ = ROWS * KT * 2 / 1024;   // glds wave-instructions per tile (all waves)
  static constexpr int NI = NJ / NWAVES;            // per wave
  static constexpr int RPI = 1024 / (2 * KT);       // INNER_K: rows per instruction
  static constexpr int LPR = KT / 8;                // INNER_K: lanes per row
  static constexpr int CPR = ROWS / 8;              // !INNER_K: 16-B chunks per k-row
  static constexpr int KPI = 64 / CPR;              // !INNER_K: k-rows per instruction
  static_assert(NI * NWAVES == NJ && NI >= 1, "tile not divisible over the waves");
  const uint16_t* p[NI];
  int kofs[NI];
  bool ok[NI];
  int64_t rowoff[NI];
  int frame0[NI], tap[NI], ch[NI];
  const uint16_t* base;
  int64_t ld;
  int T_in, Cg;

  __device__ __forceinline__ void init(const b2p_operand& o, int z1, int z2, int wave, int lane, int mn0, int MN,
                                       int kbeg) {
    const int64_t i1 = o.gather1 ? o.gather1[z1] : (int64_t)z1;
    base = static_cast<const uint16_t*>(o.ptr) + i1 * o.bs1 + (int64_t)z2 * o.bs2;
    ld = o.ld;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = wave * NI + i;
      if constexpr (INNER_K) {
        const int r = RPI * j + lane / LPR;
        const int c = (lane % LPR) ^ swz_k<KT>(r);
        const int row = mn0 + r;
        ok[i] = row < MN;
        kofs[i] = 8 * c;
        if constexpr (CONV) {
          const int T_out = o.conv_T_out;
          const int rr = ok[i] ? row : 0;
          const int b = rr / T_out, t = rr - b * T_out;
          rowoff[i] = (int64_t)b * o.conv_sample_stride;
          frame0[i] = t * o.conv_stride - o.conv_pad;
          const int k = kbeg + 8 * c;
          tap[i] = k / o.conv_Cg;
          ch[i] = k - tap[i] * o.conv_Cg;
          p[i] = base;
        } else {
          p[i] = base + (int64_t)(ok[i] ? row : 0) * ld + kbeg + 8 * c;
        }
      } else {
        const int r = KPI * j + lane / CPR;
        const int c = (lane % CPR) ^ swz_t(r);
        const int mn = mn0 + 8 * c;
        ok[i] = mn < MN;
        kofs[i] = r;
        p[i] = base + (int64_t)(kbeg + r) * ld + (ok[i] ? mn : 0);
      }
    }
    if constexpr (CONV) {
      T_in = o.conv_T_in;
      Cg = o.conv_Cg;
    }
  }

  // this wave's NI glds for the tile starting at k0 into the operand image `img`
  __device__ __forceinline__ void issue(char* img, int wave, int k0, int K) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const void* src;
      if constexpr (INNER_K && CONV) {
        const int f = frame0[i] + tap[i];
        const bool v = ok[i] && (k0 + kofs[i] < K) && f >= 0 && f < T_in;
        src = v ? (const void*)(base + rowoff[i] + (int64_t)f * ld + ch[i]) : (const void*)g_zero_page;
        ch[i] += KT;
        while (ch[i] >= Cg) { ch[i] -= Cg; ++tap[i]; }
      } else {
        const bool v = ok[i] && (k0 + kofs[i] < K);
        src = v ? (const void*)p[i] : (const void*)g_zero_page;
        p[i] += INNER_K ? (int64_t)KT : (int64_t)KT * ld;
      }
      glds16(src, (lds_t*)(img + (wave * NI + i) * 1024));
    }
  }
};

// fragment reads ------------------------------------------------------------------------------
// k-contiguous image: rows row0 .. row0+15 (lane & 15) x k = 32*kk + 8*(lane>>4) .. +7
template <int KT>
__device__ __forceinline__ bf16x8 frag_k(const char* img, int row0, int kk, int lane) {
  const int r = row0 + (lane & 15);
  const int c = (4 * kk + (lane >> 4)) ^ swz_k<KT>(r);
  return *reinterpret_cast<const bf16x8*>(img + r * (2 * KT) + c * 16);
}
// mn-contiguous image (ROWS mn-values per k-row): columns col0 .. col0+15 (lane & 15) x
// k = 32*kk + 8*(lane>>4) .. +7
template <int ROWS>
__device__ __forceinline__ bf16x8 frag_t(const char* img, int col0, int kk, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = (col0 >> 3) + (p >> 1);
  s16x4 h[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int row = 32 * kk + 8 * g + 4 * hh + q;
    const char* a = img + row * (2 * ROWS) + ((chunk ^ swz_t(row)) << 4) + 8 * (p & 1);
    h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a));
  }
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Epilogue of one 64-row band of a BN-wide output tile, staged in LDS (Cs, row stride BN + 4
// floats): every thread handles 4 consecutive columns of rows rbase, rbase + RPP, ... (16-B loads /
// stores of C, bias, aux, residual; 8-B bf16 copies) and accumulates the final values for the fused
// column sums. UNR = unroll of the row passes (0 = full): the epilogue body (bias, activations,
// dropout hash, act', residual, bf16 copies) is large, and a fully unrolled 256 x 256 epilogue
// (4 bands x 8 passes) overflowed the instruction cache (measured ~75k cycles per tile).
#ifndef B2P_EPI_UNROLL_SMALL
#define B2P_EPI_UNROLL_SMALL 0   // 0 = full unroll of the row passes
#endif
#ifndef B2P_EPI_UNROLL_PP
#define B2P_EPI_UNROLL_PP 1      // 1 = rolled
#endif
template <int BN, int NT, int UNR>
__device__ __forceinline__ void store_band(const EpiArgs& ea, const float* Cs, int tid, int z, int z1, int z2, int M,
                                           int N, float* slab, int mband, int n0, float4& csum) {
  constexpr int CG = BN / 4, RPP = NT / CG, CS_LD = BN + 4;
  const int cg = tid % CG, rbase = tid / CG;
  auto pass = [&](int i) {
    const int rl = rbase + RPP * i;
    const float4 v = *reinterpret_cast<const float4*>(Cs + rl * CS_LD + 4 * cg);
    const int m = mband + rl, n = n0 + 4 * cg;
    if (slab) {
      if (m < M) {
        float* dst = slab + (int64_t)m * N + n;
        if (ea.vec4 && n + 4 <= N) *reinterpret_cast<float4*>(dst) = v;
        else {
          if (n < N) dst[0] = v.x;
          if (n + 1 < N) dst[1] = v.y;
          if (n + 2 < N) dst[2] = v.z;
          if (n + 3 < N) dst[3] = v.w;
        }
      }
    } else {
      const float4 f = epilogue_store4(ea, z, z1, z2, m, n, v);
      csum.x += f.x; csum.y += f.y; csum.z += f.z; csum.w += f.w;
    }
  };
  if constexpr (UNR == 0) {
#pragma unroll
    for (int i = 0; i < 64 / RPP; ++i) pass(i);
  } else if constexpr (UNR == 1) {
#pragma clang loop unroll(disable)
    for (int i = 0; i < 64 / RPP; ++i) pass(i);
  } else {
#pragma unroll UNR
    for (int i = 0; i < 64 / RPP; ++i) pass(i);
  }
}

// fused bias-gradient column sums: the RPP threads of each column group add their partial sums
// (one BM-row tile partial; partial rows are 128-row granular, a 256-row tile zeroes its second row)
template <int BM, int BN, int NT>
__device__ __forceinline__ void store_colsum(const EpiArgs& ea, float* Cs, int tid, int tm, int M, int N, int n0,
                                             float4 csum) {
  constexpr int CG = BN / 4, RPP = NT / CG, CS_LD = BN + 4;
  const int cg = tid % CG, rbase = tid / CG;
  __syncthreads();
  *reinterpret_cast<float4*>(Cs + rbase * CS_LD + 4 * cg) = csum;
  __syncthreads();
  if (tid < BN && n0 + tid < N) {
    float sacc = 0.f;
#pragma unroll
    for (int r = 0; r < RPP; ++r) sacc += Cs[r * CS_LD + tid];
    const int prow = tm * (BM / 128), nprow = (M + 127) / 128;
    ea.e.colsum_part[(int64_t)prow * N + n0 + tid] = sacc;
#pragma unroll
    for (int r2 = 1; r2 < BM / 128; ++r2)
      if (prow + r2 < nprow) ea.e.colsum_part[(int64_t)(prow + r2) * N + n0 + tid] = 0.f;
  }
}

// output tile of linear tile index t: row-major (grp = 0), or grouped (grp > 0): column sweeps over
// bands of grp row tiles, so the workgroups resident on one XCD at a time share a few A row panels
// and a few B column panels in that XCD's L2 instead of cycling through all of B
// grp < 0: column bands of G = (tiles_n <= 8 ? tiles_n : ceil(tiles_n / 8)) output columns, row-major
// inside a band: the workgroups of one XCD (a contiguous range of this order, see the remap) then hold
// a G-column slice of B in their L2 while every A row panel they fetch feeds G tiles running side by side
__device__ __forceinline__ void tile_of(int t, int tiles_m, int tiles_n, int grp, int& tm, int& tn) {
  if (grp < 0) {
    const int G = tiles_n <= 8 ? tiles_n : (tiles_n + 7) / 8;
    const int per = G * tiles_m;
    const int band = t / per, r = t - band * per;
    const int gs = tiles_n - band * G < G ? tiles_n - band * G : G;
    tm = r / gs;
    tn = band * G + (r - tm * gs);
  } else if (grp > 0) {
    const int per = grp * tiles_n;
    const int g = t / per, first = g * grp;
    const int gs = tiles_m - first < grp ? tiles_m - first : grp;
    const int r = t - g * per;
    tn = r / gs;
    tm = first + (r - tn * gs);
  } else {
    tm = t / tiles_n;
    tn = t - tm * tiles_n;
  }
}

// Tile configurations: BM x BN output tile, WGM x WGN waves of WTM x 64 each ((WTM/16) x 4 MFMA tiles),
// KT-deep k-tiles, S LDS stages (S-1 tiles in flight behind counted vmcnt waits + raw barriers).
template <int BM_, int BN_, int KT_, int S_, int WTM_ = 64>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, KT = KT_, S = S_, WTM = WTM_, MI = WTM_ / 16;
  static constexpr int WGM = BM / WTM, WGN = BN / 64, NW = WGM * WGN, NT = NW * 64;
  static constexpr int STAGE = (BM + BN) * KT * 2;
  static constexpr int LDS_MAIN = S * STAGE;
  static constexpr int CS_LD = BN + 4;                          // epilogue staging row (floats)
  static constexpr int LDS_EPI = 64 * CS_LD * 4;
  static constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  static constexpr int OCC = LDS > 80 * 1024 ? 1 : 2;           // workgroups per CU
};
using CfgSmall = Cfg<128, 128, 32, 3>;   // 4 waves, 3 workgroups/CU by LDS (48 KB) and VGPRs (143)
// 256 x 128 tiles of 4 waves with 128 x 64 wave tiles (8 x 4 MFMA tiles): a quarter less operand traffic
// per FLOP than 128 x 128 (1/256 + 1/128 vs 2/128 of K per output) and 12 fragment reads per 32 MFMAs
// instead of 8 per 16; 72 KB of LDS, 2 workgroups per CU (B2P_GEMM16_TALL)
using CfgTall = Cfg<256, 128, 32, 3, 128>;
// 128 x 128 x 64 tiles, 2 stages (64 KB, 2 workgroups/CU): half the barriers per K (B2P_GEMM16_K64)
using CfgK64 = Cfg<128, 128, 64, 2>;
// Measured and removed (DESIGN.md "rejected"): 128 x 128 x 64 two-stage tiles (no gain inside the step),
// 128 x 64 tiles for N <= 1024 grids (59.3 -> 57.1 steps/s), 4-stage 128 x 128 x 32 (-10 % at K = 768),
// 256 x 128 x 64 eight-wave tiles (lock-stepped waves idle the MFMA pipe at every barrier).

// H16: the operands are fp16 (Operand.dtype 2, precision 2) and feed v_mfma_f32_16x16x32_f16; the
// data movement is the same 16-bit copy either way
template <class CF, bool AK, bool BK, bool ACONV, bool H16 = false>
__global__ void __launch_bounds__(CF::NT, CF::OCC) gemm16_kernel(const b2p_gemm_desc d, const EpiArgs ea, int tiles_m,
                                                                int tiles_n, int grp) {
  constexpr int BM = CF::BM, BN = CF::BN, KT = CF::KT, S = CF::S, NT = CF::NT;
  constexpr int A_BYTES = BM * KT * 2;
  constexpr int STAGE_BYTES = CF::STAGE;
  constexpr int CS_LD = CF::CS_LD;
  using SA = Src<BM, KT, AK, ACONV, CF::NW>;
  using SB = Src<BN, KT, BK, false, CF::NW>;
  constexpr int PT = SA::NI + SB::NI;                          // glds per wave per tile (A + B)
  __shared__ __attribute__((aligned(1024))) char smem[CF::LDS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CF::WGN, wn = wave % CF::WGN;

  // XCD-aware remap (bijective): blocks with equal blockIdx.x % 8 share an XCD and its L2, so
  // give each such group a contiguous range of tiles (neighbouring tiles share A rows).
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = tiles_m * tiles_n;
  const int zz = wgid / tiles;
  const int t = wgid - zz * tiles;
  int tm, tn;
  tile_of(t, tiles_m, tiles_n, grp, tm, tn);

  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  const int z = zz / ks, ksl = zz - z * ks;
  const int z1 = z / d.nz2, z2 = z - z1 * d.nz2;
  const int m0 = tm * BM, n0 = tn * BN;
  const int M = (int)d.M, N = (int)d.N;
  const int kchunk = ks > 1 ? (int)d.kchunk : (int)d.K;
  const int kbeg = ksl * kchunk;
  const int K = ((int)d.K < kbeg + kchunk) ? (int)d.K : kbeg + kchunk;
  const int nk = (K > kbeg && !b2p_gated_off(ea.gate)) ? (K - kbeg + KT - 1) / KT : 0;

  SA sa;
  SB sb;
  sa.init(d.A, z1, z2, wave, lane, m0, M, kbeg);
  sb.init(d.B, z1, z2, wave, lane, n0, N, kbeg);

  constexpr int MI = CF::MI;
  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: S-1 tiles in flight
#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    if (s < nk) {
      sa.issue(smem + s * STAGE_BYTES, wave, kbeg + s * KT, K);
      sb.issue(smem + s * STAGE_BYTES + A_BYTES, wave, kbeg + s * KT, K);
    }
  }
  int cur = 0;              // stage of tile kt
  int nxt = S - 1;          // stage receiving tile kt + S - 1
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's share of tile kt has landed (later tiles may stay in flight) ...
    if (kt + S - 2 < nk) wait_vm<(S - 2) * PT>();
    else wait_vm<0>();
    // ... and everyone's has; every wave is also done reading stage kt-1 (= nxt)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) {
      char* img = smem + nxt * STAGE_BYTES;
      sa.issue(img, wave, kbeg + (kt + S - 1) * KT, K);
      sb.issue(img + A_BYTES, wave, kbeg + (kt + S - 1) * KT, K);
    }
    const char* As = smem + cur * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < KT / 32; ++kk) {
      bf16x8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = BK ? frag_k<KT>(Bs, wn * 64 + j * 16, kk, lane) : frag_t<BN>(Bs, wn * 64 + j * 16, kk, lane);
      // A fragments in groups of 4 rows of MFMA tiles: at most 8 fragments live beside the
      // (MI x 4) accumulators (the 128-row wave tile would otherwise exceed 256 registers)
#pragma unroll
      for (int i0 = 0; i0 < MI; i0 += 4) {
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = AK ? frag_k<KT>(As, wm * CF::WTM + (i0 + i) * 16, kk, lane)
                     : frag_t<BM>(As, wm * CF::WTM + (i0 + i) * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if constexpr (H16)
              acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                  __builtin_bit_cast(f16x8g, af[i]), __builtin_bit_cast(f16x8g, bfr[j]), acc[i0 + i][j], 0, 0, 0);
            else
              acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i0 + i][j], 0, 0, 0);
      }
    }
    cur = cur + 1 == S ? 0 : cur + 1;
    nxt = nxt + 1 == S ? 0 : nxt + 1;
  }

  // epilogue, staged through LDS one 64-row wave band at a time
  float* Cs = reinterpret_cast<float*>(smem);
  float* slab = ks > 1 ? d.workspace + ((int64_t)z * ks + ksl) * (int64_t)M * N : nullptr;
  float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);   // fused bias-gradient column sums (colsum_part)
  constexpr int HB = CF::WTM / 64;   // 64-row bands per wave row
#pragma unroll
  for (int band = 0; band < BM / 64; ++band) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (wm == band / HB) {
      // static accumulator indices on both paths (a runtime index would move acc to scratch)
      auto stage = [&](auto hbc) {
        constexpr int hb = decltype(hbc)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              Cs[(i * 16 + (lane >> 4) * 4 + r) * CS_LD + wn * 64 + j * 16 + (lane & 15)] = acc[hb * 4 + i][j][r];
      };
      if (band % HB == 0) stage(std::integral_constant<int, 0>());
      else if constexpr (HB > 1) stage(std::integral_constant<int, 1>());
    }
    __syncthreads();
    store_band<BN, NT, B2P_EPI_UNROLL_SMALL>(ea, Cs, tid, z, z1, z2, M, N, slab, m0 + band * 64, n0, csum);
  }
  if (ea.e.colsum_part) store_colsum<BM, BN, NT>(ea, Cs, tid, tm, M, N, n0, csum);
}

// ------------------------------------------------------------------------------------------------
// 256 x 256 x 64 ping-pong kernel: 8 waves in two groups of 4 (group g owns output rows
// 128g .. 128g+127, wave wc of the group columns 64wc .. 64wc+63: a 128 x 64 sub-tile, 8 x 4 MFMA
// tiles). Every K-tile runs in 4 phases, one output quadrant (64 x 32, K 64 = 16 MFMAs) each:
//     ds_read this quadrant's fragments, [issue LDS-DMA of the next K-tile], lgkmcnt(0), barrier,
//     16 MFMAs, barrier.
// Group 1 starts one barrier later than group 0, so on every SIMD (one wave of each group) one wave
// feeds the matrix pipe while its partner reads fragments and issues DMA. Two LDS buffers: tile
// kt+1 is DMA'd into the idle buffer in phases 0 (A) and 1 (B) of tile kt and waited for
// (vmcnt(0)) in phase 3 before that phase's first barrier, so every reader of tile kt+1 passes a
// barrier after every issuer's wait. Every fragment read is retired (lgkmcnt(0)) before the
// phase's first barrier, so the buffer a DMA overwrites has no read in flight (WAR).
#ifdef B2P_PP_STAMPS   // diagnostic build only (tools/pp_probe.hip): per-workgroup clock stamps
__device__ unsigned long long g_pp_stamps[8 * 8192];
#define PP_STAMP(k)                                                                          \
  do {                                                                                       \
    if (tid == 0 && blockIdx.x < 8192) {                                                     \
      g_pp_stamps[(size_t)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime();              \
      g_pp_stamps[(size_t)blockIdx.x * 8 + 4 + (k)] = __builtin_amdgcn_s_memrealtime();      \
    }                                                                                        \
  } while (0)
#else
#define PP_STAMP(k)
#endif

constexpr int PP_NT = 512;
constexpr int PP_KT = 64;
constexpr int PP_ABYTES = 256 * PP_KT * 2;              // 32 KB per operand per buffer
constexpr int PP_STAGE = 2 * PP_ABYTES;
constexpr int PP_LDS = 2 * PP_STAGE;                    // 128 KB
constexpr int PP_CS_LD = 256 + 4;

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pp_lgkm0() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool AK, bool BK>
__global__ void __launch_bounds__(PP_NT, 1) gemm16_pp_kernel(const b2p_gemm_desc d, const EpiArgs ea, int tiles_m,
                                                            int tiles_n, int grp) {
  using SA = Src<256, PP_KT, AK, false, 8>;
  using SB = Src<256, PP_KT, BK, false, 8>;
  __shared__ __attribute__((aligned(1024))) char smem[PP_LDS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = wave >> 2, wc = wave & 3;
  PP_STAMP(0);

  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = tiles_m * tiles_n;
  const int zz = wgid / tiles;
  const int t = wgid - zz * tiles;
  int tm, tn;
  tile_of(t, tiles_m, tiles_n, grp, tm, tn);

  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  const int z = zz / ks, ksl = zz - z * ks;
  const int z1 = z / d.nz2, z2 = z - z1 * d.nz2;
  const int m0 = tm * 256, n0 = tn * 256;
  const int M = (int)d.M, N = (int)d.N;
  const int kchunk = ks > 1 ? (int)d.kchunk : (int)d.K;
  const int kbeg = ksl * kchunk;
  const int K = ((int)d.K < kbeg + kchunk) ? (int)d.K : kbeg + kchunk;
  const int nk = (K > kbeg && !b2p_gated_off(ea.gate)) ? (K - kbeg + PP_KT - 1) / PP_KT : 0;

  SA sa;
  SB sb;
  sa.init(d.A, z1, z2, wave, lane, m0, M, kbeg);
  sb.init(d.B, z1, z2, wave, lane, n0, N, kbeg);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    sa.issue(smem, wave, kbeg, K);
    sb.issue(smem + PP_ABYTES, wave, kbeg, K);
  }
  wait_vm<0>();
  pp_barrier();
  if (g == 1) pp_barrier();   // the stagger
  PP_STAMP(1);

  bf16x8 a[4][2], b[2][2];
  const int arow = g * 128, bcol = wc * 64;
  auto readA = [&](const char* As, int mi) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        a[i][kk] = AK ? frag_k<PP_KT>(As, arow + mi * 64 + i * 16, kk, lane)
                      : frag_t<256>(As, arow + mi * 64 + i * 16, kk, lane);
  };
  auto readB = [&](const char* Bs, int nj) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        b[j][kk] = BK ? frag_k<PP_KT>(Bs, bcol + nj * 32 + j * 16, kk, lane)
                      : frag_t<256>(Bs, bcol + nj * 32 + j * 16, kk, lane);
  };
  auto mfma = [&](int mi, int nj) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          acc[mi * 4 + i][nj * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b[j][kk], acc[mi * 4 + i][nj * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  for (int kt = 0; kt < nk; ++kt) {
    const char* As = smem + (kt & 1) * PP_STAGE;
    const char* Bs = As + PP_ABYTES;
    char* nx = smem + ((kt + 1) & 1) * PP_STAGE;
    const bool more = kt + 1 < nk;
    const int knext = kbeg + (kt + 1) * PP_KT;
    // phase 0: quadrant (0, 0); DMA A of tile kt+1
    readA(As, 0);
    readB(Bs, 0);
    if (more) sa.issue(nx, wave, knext, K);
    pp_lgkm0();
    pp_barrier();
    mfma(0, 0);
    pp_barrier();
    // phase 1: quadrant (0, 1); DMA B of tile kt+1
    readB(Bs, 1);
    if (more) sb.issue(nx + PP_ABYTES, wave, knext, K);
    pp_lgkm0();
    pp_barrier();
    mfma(0, 1);
    pp_barrier();
    // phase 2: quadrant (1, 1)
    readA(As, 1);
    pp_lgkm0();
    pp_barrier();
    mfma(1, 1);
    pp_barrier();
    // phase 3: quadrant (1, 0); tile kt+1 must have landed before this phase's first barrier
    readB(Bs, 0);
    wait_vm<0>();
    pp_lgkm0();
    pp_barrier();
    mfma(1, 0);
    pp_barrier();
  }
  if (g == 0) pp_barrier();   // equal barrier counts for both groups
  PP_STAMP(2);

  // epilogue: four 64-row bands through LDS (band = 2 * group + row half)
  float* Cs = reinterpret_cast<float*>(smem);
  float* slab = ks > 1 ? d.workspace + ((int64_t)z * ks + ksl) * (int64_t)M * N : nullptr;
  float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma clang loop unroll(disable)
  for (int band = 0; band < 4; ++band) {
    __syncthreads();
    if (g == (band >> 1)) {
      if (band & 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              Cs[(i * 16 + (lane >> 4) * 4 + r) * PP_CS_LD + wc * 64 + j * 16 + (lane & 15)] = acc[4 + i][j][r];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              Cs[(i * 16 + (lane >> 4) * 4 + r) * PP_CS_LD + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
      }
    }
    __syncthreads();
    store_band<256, PP_NT, B2P_EPI_UNROLL_PP>(ea, Cs, tid, z, z1, z2, M, N, slab, m0 + band * 64, n0, csum);
  }
  if (ea.e.colsum_part) store_colsum<256, 256, PP_NT>(ea, Cs, tid, tm, M, N, n0, csum);
  PP_STAMP(3);
}

}  // namespace

// row-tile band of the grouped tile order (tile_of); B2P_GEMM16_GROUP / B2P_GEMM16_GROUP_PP override
static int gemm16_group(bool pp) {
  static const int g_small = getenv("B2P_GEMM16_GROUP") ? atoi(getenv("B2P_GEMM16_GROUP")) : 0;
  static const int g_pp = getenv("B2P_GEMM16_GROUP_PP") ? atoi(getenv("B2P_GEMM16_GROUP_PP")) : 0;
  return pp ? g_pp : g_small;
}

template <class CF>
static void launch_cfg(const b2p_gemm_desc& d, const EpiArgs& ea, hipStream_t st, dim3 grid, int tm, int tn) {
  const dim3 block(CF::NT);
  const bool AK = d.A.inner_is_k != 0, BK = d.B.inner_is_k != 0;
  if (d.A.dtype == 2) {   // fp16 operands (precision 2): plain operand pairs only
    if (AK && BK) hipLaunchKernelGGL((gemm16_kernel<CF, true, true, false, true>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
    else if (AK) hipLaunchKernelGGL((gemm16_kernel<CF, true, false, false, true>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
    else hipLaunchKernelGGL((gemm16_kernel<CF, false, false, false, true>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
    return;
  }
  if (AK && BK) {
    if (d.A.conv) hipLaunchKernelGGL((gemm16_kernel<CF, true, true, true>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
    else hipLaunchKernelGGL((gemm16_kernel<CF, true, true, false>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
  } else if (AK && !BK) {
    if (d.A.conv) hipLaunchKernelGGL((gemm16_kernel<CF, true, false, true>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
    else hipLaunchKernelGGL((gemm16_kernel<CF, true, false, false>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
  } else {
    hipLaunchKernelGGL((gemm16_kernel<CF, false, false, false>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(false));
  }
}

int b2p_gemm16_launch(const b2p_gemm_desc& d, hipStream_t st) {
  const EpiArgs ea = make_epi_args(d);
  if ((d.ep.colsum_part || d.ep.pre16 || d.ep.aux16) && !ea.vec4) {
    b2p_set_error("gemm16: colsum_part / pre16 / aux16 need 16-B aligned C-shaped tensors and N %% 4 == 0");
    return 1;
  }
  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  const int64_t nz = (int64_t)d.nz1 * d.nz2 * ks;
  const bool h16 = d.A.dtype == 2;
  if (h16 && d.A.conv) {
    b2p_set_error("gemm16: fp16 operands support plain (non-conv) views only");
    return 1;
  }
  // 256 x 256 ping-pong tile (B2P_GEMM16_PP: 0 off, 1 (default) for long-K launches whose grid fills
  // most of the chip, 2 always for plain operands). One workgroup per CU cannot hide its epilogue
  // behind another tile's K loop, so at K <= 1024 (the encoder's projections, 2-3 tiles per CU
  // with the 128 x 128 kernel) it measured slower; at K >= 2048 its K loop (~1.0 PF) wins, and so
  // does a split-K launch of >= 1024-deep slices (the weight gradients, K = tokens).
  static int pp_mode = getenv("B2P_GEMM16_PP") ? atoi(getenv("B2P_GEMM16_PP")) : 1;
  const int64_t tiles_pp = ((d.M + 255) / 256) * ((d.N + 255) / 256) * nz;
  const int64_t kper = ks > 1 ? (int64_t)d.kchunk : d.K;
  const bool pp = !h16 && !d.A.conv && (pp_mode == 2 || (pp_mode == 1 && ((tiles_pp >= 192 && kper >= 2048) || (ks > 1 && tiles_pp >= 160 && kper >= 1024))));
  if (pp) {
    const int tm = (int)((d.M + 255) / 256), tn = (int)((d.N + 255) / 256);
    const dim3 grid((unsigned)tiles_pp), block(PP_NT);
    const bool AK = d.A.inner_is_k != 0, BK = d.B.inner_is_k != 0;
    if (AK && BK) hipLaunchKernelGGL((gemm16_pp_kernel<true, true>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(true));
    else if (AK) hipLaunchKernelGGL((gemm16_pp_kernel<true, false>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(true));
    else hipLaunchKernelGGL((gemm16_pp_kernel<false, false>), grid, block, 0, st, d, ea, tm, tn, gemm16_group(true));
    return 0;
  }
  const int tm = (int)((d.M + 127) / 128), tn = (int)((d.N + 127) / 128);
  const int64_t nwg = (int64_t)tm * tn * nz;
  if (nwg >= (1ll << 31)) {
    b2p_set_error("gemm16: grid too large");
    return 1;
  }
  if (ks > 1 && d.kchunk % 32 != 0) {
    b2p_set_error("gemm16: split-K chunk must be a multiple of 32");
    return 1;
  }
  // 256 x 128 tiles (B2P_GEMM16_TALL: 0 off, 1 when the grid still gives every CU at least `tall_min`
  // tiles of 256 x 128, default 2): plain or conv operands, any split
  static int tall = getenv("B2P_GEMM16_TALL") ? atoi(getenv("B2P_GEMM16_TALL")) : 0;
  static int tall_min = getenv("B2P_GEMM16_TALL_MIN") ? atoi(getenv("B2P_GEMM16_TALL_MIN")) : 512;
  const int tmt = (int)((d.M + 255) / 256);
  const int64_t nwg_t = (int64_t)tmt * tn * nz;
  if (tall && nwg_t >= tall_min) {
    launch_cfg<CfgTall>(d, ea, st, dim3((unsigned)nwg_t), tmt, tn);
    return 0;
  }
  // 128 x 128 x 64 two-stage tiles (B2P_GEMM16_K64: 0 never = default, 1 always, -1 for grids of < 512
  // tiles). In isolation (tools/gemm_ab.py, L2-warm repeated launches; profiles/r03s_gemm_k64_ab.txt)
  // the N = 768 encoder shapes and the 768 x 768 split-K weight gradient ran 7-15 % faster with -1, but
  // inside the step (cold operands, side-stream concurrency) base and Conformer steps did not move
  // (16.46 vs 16.44 ms, 88.2 vs 88.6 ms; profiles/r03t_k64_step_ab.txt), so the default stays off.
  static int k64 = getenv("B2P_GEMM16_K64") ? atoi(getenv("B2P_GEMM16_K64")) : 0;
  if ((k64 == 1 || (k64 < 0 && nwg < 512)) && (ks == 1 || d.kchunk % 64 == 0)) {
    launch_cfg<CfgK64>(d, ea, st, dim3((unsigned)nwg), tm, tn);
    return 0;
  }
  launch_cfg<CfgSmall>(d, ea, st, dim3((unsigned)nwg), tm, tn);
  return 0;
}
