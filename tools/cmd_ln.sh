set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ln; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
tail -1 $O/b.json | cut -c1-220
timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --steps 10 --warmup 3 > $O/c.json 2> $O/c.err || { tail -5 $O/c.err; exit 1; }
tail -1 $O/c.json | cut -c1-220
