set -u
# Round-2 re-entry check of HEAD: GPU parity suite, smoke(), base and Conformer bench lines.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_conf.json 2> $O/bench_conf.err || { tail -20 $O/bench_conf.err; exit 1; }
tail -1 $O/bench_conf.json
