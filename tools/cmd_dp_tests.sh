set -u
# data-parallel and trainer GPU tests in one process. usage: bash tools/cmd_dp_tests.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dp_tests}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_trainer_gpu.py tests/test_dp_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "worst relative|passed|failed|Error" $O/tests.log | tail -8
exit $rc
