set -u
# GPU tests only (prebuilt library): bash tools/cmd_tests.sh <tag> [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tests}
mkdir -p $O
K=${2:-}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 \
  || { tail -80 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -3
