set -u
# GPU tests only (prebuilt library): bash tools/cmd_tests.sh <tag> [pytest -k expr] [extra pytest args]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tests}
mkdir -p $O
K=${2:-}
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${3:-} ${K:+-k "$K"} > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -60
tail -3 $O/pytest.log
exit $rc
