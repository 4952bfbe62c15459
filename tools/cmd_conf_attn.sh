set -u
# Conformer fused attention check: Conformer GPU tests, bs=32 bf16 loss error, then the bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/conf_attn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "conf or rotary" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/bf16_err.py conformer 32 > $O/bf16_err.log 2>&1 || { tail -20 $O/bf16_err.log; exit 1; }
tail -1 $O/bf16_err.log
timeout -k 10 400 python bench.py --config conformer --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
