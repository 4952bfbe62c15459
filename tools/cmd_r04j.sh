set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_configs34_gpu.py tests/test_model_gpu.py -v -s --timeout 300 --timeout-method thread > $O/pytest2.log 2>&1
rc=$?
grep -E "FAILED|rel \[|worst relative|passed|failed" $O/pytest2.log | tail -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python -u tools/traj_err.py base 3 "-" > $O/traj_base.log 2>&1; grep "^.base" $O/traj_base.log
