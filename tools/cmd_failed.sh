set -u
# rerun a list of GPU test node ids with tracebacks: bash tools/cmd_failed.sh <tag> <nodeid>...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --tb=short --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -40
exit $rc
