set -u
# Round-2 final profile of the current tree: GPU suite, smoke(), default bench line (with CPU baseline),
# Conformer bench line, rocprofv3 kernel stats of the base bench (replayed-step breakdown).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAIL|Error" $O/pytest.log | tail -20; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_conf.json 2> $O/bench_conf.err || { tail -20 $O/bench_conf.err; exit 1; }
tail -1 $O/bench_conf.json
P=$O/prof; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $P/prof.log 2>&1 || { tail -20 $P/prof.log; exit 1; }
tail -1 $P/prof.log
python tools/step_breakdown.py $P 6 45 > $O/base_replay_step.txt 2>&1 || true
head -12 $O/base_replay_step.txt
P2=$O/prof_conf; mkdir -p $P2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P2 -o run -- python3 bench.py --config conformer --steps 6 --warmup 2 --no-cpu-baseline --no-parity > $P2/prof.log 2>&1 || { tail -20 $P2/prof.log; exit 1; }
python tools/step_breakdown.py $P2 4 45 > $O/conformer_replay_step.txt 2>&1 || true
head -12 $O/conformer_replay_step.txt
