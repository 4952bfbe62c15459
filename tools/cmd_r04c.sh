set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|rel \[|worst relative" $O/pytest.log | tail -30
tail -3 $O/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab.log 2>&1 && tail -12 $O/gemm_ab.log
B2P_GEMM16_PP=2 timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab_pp.log 2>&1 && tail -12 $O/gemm_ab_pp.log
timeout -k 10 200 python -u tools/gemm_vs_blas.py > $O/gemm_vs_blas.log 2>&1; tail -12 $O/gemm_vs_blas.log
