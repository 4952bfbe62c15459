// gemm16 instantiations: fp16 operands, A and B k-contiguous
#include "gemm16_impl.inc"

int gemm16_run_nt_f16(const b2p_gemm_desc& d, hipStream_t st, int fam, uint32_t ek, unsigned nwg, int tm, int tn, int grp,
                      uint32_t* ctr) {
  EpiArgs ea = make_epi_args(d);
  ea.rk = ek;   // EK_RUNTIME instantiations read the kind bits at run time
  ea.tile_ctr = ctr;   // split-K fix-up counters (nullptr: the separate reduce launch)
  const bool AK = d.A.inner_is_k != 0, BK = d.B.inner_is_k != 0;
  if (!(AK && BK)) { b2p_set_error("gemm16: internal dispatch"); return 1; }
  if (fam == G16_PP) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_pp<true, true, true, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_F16(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_pp<true, true, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_pp<true, true, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_PP192) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_pp192<true, true, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_F16(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_pp192<true, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_pp192<true, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_PN256 || fam == G16_PN192) {
    const bool w = fam == G16_PN256;
    switch (ek) {
#define B2P_GO_(K) case K: if (w) launch_pn<256, true, K>(d, ea, st, nwg, tm, tn, grp); else launch_pn<192, true, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_F16(B2P_GO_)
#undef B2P_GO_
      default: if (w) launch_pn<256, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); else launch_pn<192, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_SMALL) {
    switch (ek) {
#define B2P_GO_(K) case K: launch_small<CfgSmall, true, true, false, true, K>(d, ea, st, nwg, tm, tn, grp); return 0;
      B2P_KINDS_NT_F16(B2P_GO_)
#undef B2P_GO_
      default: if (ek == EK_GENERIC) launch_small<CfgSmall, true, true, false, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp); else launch_small<CfgSmall, true, true, false, true, EK_RUNTIME>(d, ea, st, nwg, tm, tn, grp); return 0;
    }
  }
  if (fam == G16_TALL) launch_small<CfgTall, true, true, false, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp);
  else launch_small<CfgK64, true, true, false, true, EK_GENERIC>(d, ea, st, nwg, tm, tn, grp);
  return 0;
}
