// gemm16 instantiations: bf16 operands, A and B k-contiguous
#include "gemm16_impl.inc"

int gemm16_run_nt_bf16(const b2p_gemm_desc& d, hipStream_t st, int fam, uint32_t ek, unsigned nwg, int tm, int tn, int grp,
                      uint32_t* ctr) {
  EpiArgs ea = make_epi_args(d);
  ea.rk = ek;   // EK_RUNTIME instantiations read the kind bits at run time
  ea.tile_ctr = ctr;   // split-K fix-up counters (nullptr: the separate reduce launch)
  if (fam == G16_PP) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_pp<true, true, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_BF16(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_pp<true, true, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_pp<true, true, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_PP192) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_pp192<true, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_BF16(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_pp192<true, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_pp192<true, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_PN256 || fam == G16_PN192) {
    const bool w = fam == G16_PN256;
    switch (ek) {
#define B2P_GO_(K) case K: if (w) launch_pn<256, false, K>(d, ea, st, nwg, tm, tn, grp); else launch_pn<192, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_BF16(B2P_GO_)
#undef B2P_GO_
      default: if (w) launch_pn<256, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); else launch_pn<192, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_SMALL) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_small<CfgSmall, true, true, false, false, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_BF16(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_small<CfgSmall, true, true, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, true, true, false, false, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_TALL) launch_small<CfgTall, true, true, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp);
  else launch_small<CfgK64, true, true, false, false, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp);
  return 0;
}
