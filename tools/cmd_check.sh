set -u
# GPU check of the current tree with its prebuilt library: pytest -m gpu, then the default bench line.
# usage: bash tools/cmd_check.sh <tag> [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-check}
mkdir -p $O
K=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 \
  || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 500 python bench.py --gpus 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
