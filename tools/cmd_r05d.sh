set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d; mkdir -p $O
B2P_GEMM16_P4=1 B2P_GEMM16_PP=2 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests_p4.log 2>&1
rc=$?; tail -3 $O/gemm_tests_p4.log; [ $rc -ne 0 ] && exit $rc
B2P_GEMM16_PP=2 timeout -k 10 400 python -u tools/p4_ab.py 5 > $O/p4_ab.txt 2>&1; rc=$?; cat $O/p4_ab.txt; exit $rc
