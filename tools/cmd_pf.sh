set -u
# prefetch K-loop check: gemm tests, then gemm_ab with B2P_GEMM16_PF=1 (default) and 0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pf}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab.log 2>&1 && tail -16 $O/gemm_ab.log
B2P_GEMM16_PF=0 timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab_pf0.log 2>&1 && tail -16 $O/gemm_ab_pf0.log
