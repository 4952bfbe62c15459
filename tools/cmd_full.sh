set -u
# full GPU suite + the default bench line: bash tools/cmd_full.sh <tag> [pytest -k expression]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-full}
mkdir -p $O
K=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|rel \[|worst relative" $O/pytest.log | tail -30
tail -3 $O/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; rc2=$?
tail -c 3000 $O/bench.log
exit $rc2
