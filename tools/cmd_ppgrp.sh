set -u
# ping-pong tile order (B2P_GEMM16_GROUP_PP) and B-DMA placement (probe_bin/pp_probe_be) A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ppgrp}
mkdir -p $O
export B2P_GEMM16_PP=2
for s in "8192 8192 8192 0 0" "7968 3072 768 1 0" "7968 4096 1024 1 0"; do
  for g in 0 4 8 -1; do
    echo "== GROUP_PP=$g $s"
    B2P_GEMM16_GROUP_PP=$g timeout -k 5 60 ./probe_bin/pp_probe $s || exit 1
  done
  echo "== B_EARLY $s"
  timeout -k 5 60 ./probe_bin/pp_probe_be $s || exit 1
done > $O/ppgrp.log 2>&1
grep -E "==|us/launch|k-loop|epilogue|clock" $O/ppgrp.log
