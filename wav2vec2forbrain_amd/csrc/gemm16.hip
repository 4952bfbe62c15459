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
#include "gemm16_impl.inc"
#include <algorithm>

// row-tile band of the grouped tile order (tile_of); B2P_GEMM16_GROUP / B2P_GEMM16_GROUP_PP override
static int gemm16_group(bool pp) {
  static const int g_small = getenv("B2P_GEMM16_GROUP") ? atoi(getenv("B2P_GEMM16_GROUP")) : 0;
  static const int g_pp = getenv("B2P_GEMM16_GROUP_PP") ? atoi(getenv("B2P_GEMM16_GROUP_PP")) : 0;
  return pp ? g_pp : g_small;
}

// epilogue kind of a launch (gemm16_impl.inc: EK_*); EK_GENERIC where the fast kinds' assumptions fail
static uint32_t epi_kind(const b2p_gemm_desc& d, const EpiArgs& ea) {
  if (d.ksplit > 1) return EK_SLAB;
  const b2p_epilogue& e = d.ep;
  // vectorised accesses, no gathered bias, 32-bit byte offsets
  const int64_t ldmax = std::max({e.ldc, e.ldr, e.ldaux, (int64_t)1});
  if (!ea.vec4 || e.bias_gather || (d.M * ldmax + d.N) * 4 >= 0xFFFFFFF0ll) return EK_GENERIC;
  uint32_t k = 0;
  if (e.beta != 0.f) k |= EK_BETA;
  if (e.bias) k |= EK_BIAS;
  if (e.pre_out) k |= EK_PRE32;
  if (e.pre16) k |= EK_PRE16;
  if (e.act != B2P_ACT_NONE) k |= EK_ACT;
  if (e.drop_p > 0.f) k |= EK_DROP;
  if (e.act_bwd != B2P_ACT_NONE) k |= EK_ABWD | (e.aux16 ? EK_AUX16 : 0u);
  if (e.residual) k |= EK_RES;
  if (e.C) k |= EK_C32;
  if (e.C16) k |= EK_C16 | ((e.flags & B2P_EPI_C16_FP16) ? EK_C16H : 0u);
  if (e.colsum_part) k |= EK_CSUM;
  if (e.C16b) k |= EK_C16B;
  return k;
}

// split-K fix-up inside the GEMM (splitk_fixup, gemm16_impl.inc) instead of the reduce launch: the
// vectorised layouts, a workspace with room for one counter per 128 x 128 output tile behind the
// slabs (functional.gemm allocates it), B2P_SPLITK_FUSED=1. Off by default: the last workgroup of a
// tile sums all its slices alone, so the weight-gradient grids (36-144 tiles x 4-7 slices) end in a
// tail of a few busy CUs: 768x768x7968 38.0 -> 64.5 us, 3072x768x7968 75.6 -> 84.0 us against the
// reduce launch spread over the chip (profiles/r04w_splitk_fused_ab.txt).
bool gemm16_splitk_fused(const b2p_gemm_desc& d) {
  static const int on = getenv("B2P_SPLITK_FUSED") ? atoi(getenv("B2P_SPLITK_FUSED")) : 0;
  if (!on || d.ksplit <= 1 || !d.workspace) return false;
  const b2p_epilogue& e = d.ep;
  const bool v4 = d.N % 4 == 0 && e.ldc % 4 == 0 && e.cbs1 % 4 == 0 && e.cbs2 % 4 == 0 &&
                  ((uintptr_t)e.C & 15u) == 0 && ((uintptr_t)e.C16 & 7u) == 0 && ((uintptr_t)d.workspace & 15u) == 0;
  const int64_t nz = (int64_t)d.nz1 * d.nz2;
  const int64_t need = (int64_t)d.ksplit * nz * d.M * d.N + ((d.M + 127) / 128) * ((d.N + 127) / 128) * nz;
  return v4 && d.workspace_floats >= need;
}

// Kernel variant knob (b2p_gemm16_variant, B2P_GEMM16_VARIANT; A/B tools), bits: 1 = the 256-column ping-pong
// kernel without the quarter-scheduled DMA, 2 = no narrow ping-pong kernel (those launches on 128 x 128)
static int g_variant = getenv("B2P_GEMM16_VARIANT") ? atoi(getenv("B2P_GEMM16_VARIANT")) : 0;
int gemm16_variant_get() { return g_variant; }
extern "C" int b2p_gemm16_variant(int v) {
  const int old = g_variant;
  if (v >= 0) g_variant = v;
  return old;
}

static int run(const b2p_gemm_desc& d, hipStream_t st, int fam, uint32_t ek, unsigned nwg, int tm, int tn, int grp) {
  const bool AK = d.A.inner_is_k != 0, BK = d.B.inner_is_k != 0;
  uint32_t* ctr = nullptr;
  if (gemm16_splitk_fused(d)) {
    const int64_t nz = (int64_t)d.nz1 * d.nz2;
    ctr = reinterpret_cast<uint32_t*>(d.workspace + (int64_t)d.ksplit * nz * d.M * d.N);
    if (hipMemsetAsync(ctr, 0, (size_t)tm * tn * nz * sizeof(uint32_t), st) != hipSuccess) {
      b2p_set_error("gemm16: split-K counter reset failed");
      return 1;
    }
  }
  if (AK && BK && !d.A.conv && d.A.dtype == 1) return gemm16_run_nt_bf16(d, st, fam, ek, nwg, tm, tn, grp, ctr);
  if (AK && BK && d.A.dtype == 2) return gemm16_run_nt_f16(d, st, fam, ek, nwg, tm, tn, grp, ctr);
  return gemm16_run_other(d, st, fam, ek, nwg, tm, tn, grp, ctr);
}

int b2p_gemm16_launch(const b2p_gemm_desc& d, hipStream_t st) {
  const EpiArgs ea = make_epi_args(d);
  if ((d.ep.colsum_part || d.ep.pre16 || d.ep.aux16 || d.ep.C16b) && !ea.vec4) {
    b2p_set_error("gemm16: colsum_part / pre16 / aux16 / C16b need 16-B aligned C-shaped tensors and N %% 4 == 0");
    return 1;
  }
  const int ks = d.ksplit > 1 ? d.ksplit : 1;
  const int64_t nz = (int64_t)d.nz1 * d.nz2 * ks;
  const bool h16 = d.A.dtype == 2;
  uint32_t ek = epi_kind(d, ea);
  // fused column sums only in their instantiated kinds (bf16, k-contiguous); anything else takes the
  // LDS-staged epilogue, so the runtime-kind kernels carry no column-sum code
  if ((ek & EK_CSUM) && !(d.A.inner_is_k && d.B.inner_is_k && d.A.dtype != 2 && (ek == K_GDH16CS || ek == K_GDH32CS)))
    ek = EK_GENERIC;
  if (ea.gates && !(ek == K_F || ek == K_FB || ek == K_SLAB)) {
    b2p_set_error("gemm16: per-member gates need a plain (C or beta) epilogue");
    return 1;
  }
  if (h16 && d.A.conv) {
    b2p_set_error("gemm16: fp16 operands support plain (non-conv) views only");
    return 1;
  }
  // 256 x 256 ping-pong tile (B2P_GEMM16_PP: 0 off, 1 (default) for long-K launches whose grid fills
  // most of the chip, 2 always for plain operands). One workgroup per CU cannot hide its epilogue
  // behind another tile's K loop, so at K <= 1024 (the encoder's projections, 2-3 tiles per CU
  // with the 128 x 128 kernel) it measured slower; at K >= 2048 its K loop (~1.0 PF) wins, and so
  // does a split-K launch of >= 1024-deep slices (the weight gradients, K = tokens).
  // Round 4 (register epilogue, tools/gemm_ab.py): a k-contiguous launch of >= 360 256 x 256 tiles (~1.5
  // rounds of the CUs: N >= 3072 at 7968 tokens) also runs faster on it, at K = 768 / 1024
  // (B2P_GEMM16_PP_TILES).
  static int pp_mode = getenv("B2P_GEMM16_PP") ? atoi(getenv("B2P_GEMM16_PP")) : 1;
  static int pp_tiles = getenv("B2P_GEMM16_PP_TILES") ? atoi(getenv("B2P_GEMM16_PP_TILES")) : 360;
  const int64_t tiles_pp = ((d.M + 255) / 256) * ((d.N + 255) / 256) * nz;
  const int64_t kper = ks > 1 ? (int64_t)d.kchunk : d.K;
  const bool nt = d.A.inner_is_k && d.B.inner_is_k;
  // the 256-column kernels address each operand through a raw buffer resource with 32-bit offsets
  // (SrcB, gemm16_impl.inc): every operand extent below 2^30 bytes
  auto ext_ok = [&](const b2p_operand& o, int64_t mn) {
    const int64_t rows = o.inner_is_k ? mn : d.K, cols = o.inner_is_k ? d.K : mn;
    return ((rows - 1) * o.ld + cols) * 2 < (1ll << 30);
  };
  const bool pp = !d.A.conv && (!h16 || nt) && ext_ok(d.A, d.M) && ext_ok(d.B, d.N) &&
                  (pp_mode == 2 || (pp_mode == 1 && ((tiles_pp >= 192 && kper >= 2048) ||
                                                     (ks > 1 && tiles_pp >= 160 && kper >= 1024) ||
                                                     (nt && tiles_pp >= pp_tiles && kper >= 512))));
  if (pp) {
    const int tm = (int)((d.M + 255) / 256), tn = (int)((d.N + 255) / 256);
    // 192 x 256 tiles (B2P_GEMM16_PP192: 0 off, 1 (default) when fewer rounds of the 256 CUs x tile rows
    // come out at least 8 % lower, 2 always): k-contiguous A
    static int pp192 = getenv("B2P_GEMM16_PP192") ? atoi(getenv("B2P_GEMM16_PP192")) : 1;
    if (pp192 && nt) {
      const int tm3 = (int)((d.M + 191) / 192);
      const int64_t t3 = (int64_t)tm3 * tn * nz;
      const int64_t cost256 = (tiles_pp + 255) / 256 * 256, cost192 = (t3 + 255) / 256 * 192;
      if (pp192 == 2 || cost192 * 100 <= cost256 * 92)
        return run(d, st, G16_PP192, ek, (unsigned)t3, tm3, tn, gemm16_group(true));
    }
    return run(d, st, G16_PP, ek, (unsigned)tiles_pp, tm, tn, gemm16_group(true));
  }
  // narrow ping-pong tiles, PBM x 128 (B2P_GEMM16_PN: 0 off, 1 (default) for k-contiguous launches with
  // N <= B2P_GEMM16_PN_MAX_N, 2 for every k-contiguous launch): 192 rows where fewer CU-rounds x tile rows come out of it
  // (N = 768: 252 tiles in one round), else 256 (N = 1024: 256 tiles); the LDS-staged (GENERIC) epilogue
  // stays on the other kernels
  // N <= 2048 (round 6, tools/gemm_ab.py, profiles/r06o_pn_wide_ab.txt): the Conformer's pointwise conv 1
  // (7968 x 2048 x 1024) 56.2 -> 49.8 us; the QKV projection (N = 2304) is slower on it (53.8 -> 57.2 us)
  static int pn_mode = getenv("B2P_GEMM16_PN") ? atoi(getenv("B2P_GEMM16_PN")) : 1;
  static int pn_max_n = getenv("B2P_GEMM16_PN_MAX_N") ? atoi(getenv("B2P_GEMM16_PN_MAX_N")) : 2048;
  if (pn_mode && !(gemm16_variant_get() & 2) && nt && !d.A.conv && ek != EK_GENERIC && ext_ok(d.A, d.M) && ext_ok(d.B, d.N) &&
      (ks == 1 || d.kchunk % 64 == 0) && (pn_mode == 2 || d.N <= pn_max_n)) {
    const int tn = (int)((d.N + 127) / 128), tm2 = (int)((d.M + 255) / 256), tm3 = (int)((d.M + 191) / 192);
    const int64_t t256 = (int64_t)tm2 * tn * nz, t192 = (int64_t)tm3 * tn * nz;
    const int64_t cost256 = (t256 + 255) / 256 * 256, cost192 = (t192 + 255) / 256 * 192;
    if (cost192 < cost256) return run(d, st, G16_PN192, ek, (unsigned)t192, tm3, tn, gemm16_group(true));
    return run(d, st, G16_PN256, ek, (unsigned)t256, tm2, tn, gemm16_group(true));
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
  if (tall && nwg_t >= tall_min && !h16 && nt) {
    return run(d, st, G16_TALL, ek, (unsigned)nwg_t, tmt, tn, gemm16_group(false));
  }
  // 128 x 128 x 64 two-stage tiles (B2P_GEMM16_K64: 0 never = default, 1 always, -1 for grids of < 512
  // tiles). In isolation (tools/gemm_ab.py, L2-warm repeated launches; profiles/r03s_gemm_k64_ab.txt)
  // the N = 768 encoder shapes and the 768 x 768 split-K weight gradient ran 7-15 % faster with -1, but
  // inside the step (cold operands, side-stream concurrency) base and Conformer steps did not move
  // (16.46 vs 16.44 ms, 88.2 vs 88.6 ms; profiles/r03t_k64_step_ab.txt), so the default stays off.
  static int k64 = getenv("B2P_GEMM16_K64") ? atoi(getenv("B2P_GEMM16_K64")) : 0;
  if ((k64 == 1 || (k64 < 0 && nwg < 512)) && (ks == 1 || d.kchunk % 64 == 0) && !h16 && nt) {
    return run(d, st, G16_K64, ek, (unsigned)nwg, tm, tn, gemm16_group(false));
  }
  return run(d, st, G16_SMALL, ek, (unsigned)nwg, tm, tn, gemm16_group(false));
}
