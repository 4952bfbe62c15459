set -u
# Conformer producer-written 16-bit operands: GPU suite, then base + Conformer bench lines (+ tile-order A/B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_conf.json 2> $O/bench_conf.err || { tail -20 $O/bench_conf.err; exit 1; }
tail -1 $O/bench_conf.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
B2P_GEMM16_GROUP=8 timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > $O/bench_g8.json 2> $O/bench_g8.err || { tail -20 $O/bench_g8.err; exit 1; }
tail -1 $O/bench_g8.json
