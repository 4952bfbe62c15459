set -u
# worst gradient errors of the golden step tests (for the gates), at HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py -k test_step_matches_reference_golden > $O/tests.log 2>&1; rc=$?
grep -E "worst gradient|passed|failed" $O/tests.log
exit $rc
