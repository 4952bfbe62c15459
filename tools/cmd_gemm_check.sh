set -u
# GEMM correctness + per-shape timing: bash tools/cmd_gemm_check.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gemm}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab.log 2>&1 && tail -16 $O/gemm_ab.log
B2P_GEMM16_PP=2 B2P_GEMM16_PP192=0 timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab_pp.log 2>&1 && tail -16 $O/gemm_ab_pp.log
B2P_GEMM16_PP=2 B2P_GEMM16_PP192=2 timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab_pp192.log 2>&1 && tail -16 $O/gemm_ab_pp192.log
export B2P_GEMM16_PP=2
for s in "7968 768 768 0 0" "7968 768 3072 0 0" "7968 3072 768 2 1" "7968 3072 768 1 0" "8192 8192 8192 0 0"; do timeout -k 5 60 ./probe_bin/pp_probe $s || break; done > $O/pp.log 2>&1; grep -E "us/launch|k-loop|epilogue" $O/pp.log
