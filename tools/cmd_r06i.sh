set -u
# ping-pong K-loop ablation (tools/pp_probe.hip, PP_DIAG bits: 1 no DMA, 2 no MFMA, 4 no fragment reads),
# the weight-gradient (TN) layout beside the quarter-scheduled NT one
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i; mkdir -p $O
export B2P_GEMM16_PP=2
for s in "4096 4096 7968 0 0 1" "8192 4096 7968 0 0 1" "8192 8192 8192 0 0 0" "7968 3072 768 1 0 0"; do
  for dg in 0 1 2 4 3 5 6 7; do
    echo "== PP_DIAG=$dg $s"
    PP_DIAG=$dg timeout -k 5 60 ./probe_bin/pp_probe $s || exit 1
  done
done > $O/ppdiag.log 2>&1
grep -E "==|us/launch|k-loop" $O/ppdiag.log
