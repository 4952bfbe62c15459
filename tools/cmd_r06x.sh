set -u
# LayerDrop select in place (a kept layer's select moves no bytes): LayerDrop / trainer / model / trajectory
# tests, the DP tests (reported), step A/B against B2P_LD_INPLACE=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_layerdrop_gpu.py tests/test_trainer_gpu.py tests/test_model_gpu.py tests/test_configs34_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_dp_gpu.py > $O/tests_dp.log 2>&1; rc=$?
grep -E "worst relative|passed|failed" $O/tests_dp.log | tail -12
[ $rc -gt 1 ] && exit $rc
B2P_LD_INPLACE=0 timeout -k 10 300 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_dp_gpu.py -k rccl > $O/tests_dp_off.log 2>&1
grep -E "worst relative|passed|failed" $O/tests_dp_off.log | tail -6
bash tools/cmd_ab_env.sh r06x_step "B2P_LD_INPLACE=0" || exit 1
