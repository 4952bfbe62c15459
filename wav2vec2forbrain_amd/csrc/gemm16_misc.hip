// gemm16 instantiations: the other layouts (m/n-contiguous operands, conv views)
#include "gemm16_impl.inc"

int gemm16_run_other(const b2p_gemm_desc& d, hipStream_t st, int fam, uint32_t ek, unsigned nwg, int tm, int tn, int grp,
                      uint32_t* ctr) {
  EpiArgs ea = make_epi_args(d);
  ea.rk = ek;   // EK_RUNTIME instantiations read the kind bits at run time
  ea.tile_ctr = ctr;   // split-K fix-up counters (nullptr: the separate reduce launch)
  const bool AK = d.A.inner_is_k != 0, BK = d.B.inner_is_k != 0;
  const bool h16 = d.A.dtype == 2;
  if (AK && BK) {   // bf16 with an implicit conv view on A
    if (fam == G16_TALL) { if (ek == EK_GENERIC) launch_small<CfgTall, true, true, true, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgTall, true, true, true, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); }
    else if (fam == G16_K64) { if (ek == EK_GENERIC) launch_small<CfgK64, true, true, true, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgK64, true, true, true, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); }
    else { if (ek == EK_GENERIC) launch_small<CfgSmall, true, true, true, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, true, true, true, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); }
    return 0;
  }
  if (AK && h16) { if (ek == EK_GENERIC) launch_small<CfgSmall, true, false, false, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, true, false, false, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0; }
  if (h16) { if (ek == EK_GENERIC) launch_small<CfgSmall, false, false, false, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, false, false, false, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0; }
  if (AK) {
    if (fam == G16_PP) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_pp<true, false, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_OTHER(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_pp<true, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_pp<true, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
    }
    if (d.A.conv) { if (ek == EK_GENERIC) launch_small<CfgSmall, true, false, true, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, true, false, true, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0; }
    switch (ek) {
#define B2P_GO_(K) case K: launch_small<CfgSmall, true, false, false, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_OTHER(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) { if (ek == EK_GENERIC) launch_small<CfgSmall, true, false, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, true, false, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); } else launch_small<CfgSmall, true, false, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_PP) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_pp<false, false, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_OTHER(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_pp<false, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_pp<false, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
    switch (ek) {
#define B2P_GO_(K) case K: launch_small<CfgSmall, false, false, false, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_OTHER(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) { if (ek == EK_GENERIC) launch_small<CfgSmall, false, false, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, false, false, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); } else launch_small<CfgSmall, false, false, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  return 0;
}
