set -u
# ping-pong K-loop ablation (tools/pp_probe.hip, PP_DIAG bits: 1 no DMA, 2 no MFMA, 4 no fragment reads)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ppdiag}
mkdir -p $O
export B2P_GEMM16_PP=2
for s in "8192 8192 8192 0 0" "7968 3072 768 1 0"; do
  for dg in 0 1 2 4 3 5 6 7; do
    echo "== PP_DIAG=$dg $s"
    PP_DIAG=$dg timeout -k 5 60 ./probe_bin/pp_probe $s || exit 1
  done
done > $O/ppdiag.log 2>&1
grep -E "==|us/launch|k-loop|epilogue" $O/ppdiag.log
