set -u
# ring kernel: GEMM tests with it on, then the interleaved A/B against the 2-buffer kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b; mkdir -p $O
B2P_GEMM16_RING=1 timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_wgrad_batch_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | tail; exit $rc; }
B2P_GEMM16_PP=2 timeout -k 10 300 python -u tools/ring_ab.py 5 > $O/ring_ab.txt 2>&1; rc=$?; cat $O/ring_ab.txt; exit $rc
