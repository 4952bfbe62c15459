set -u
# full GPU suite on the round-6 tree, attention bench, base / Conformer bench lines, Conformer replay step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | tail; exit $rc; }
timeout -k 10 120 python3 tools/attn_bench.py > $O/attn_bench.txt 2>&1 || { tail -5 $O/attn_bench.txt; exit 1; }; grep attn16 $O/attn_bench.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('base', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['max_rel_err'])
c=d['conformer_large']; print('conformer', c['value'], c['ms_per_step'], c['roofline']['frac'], c['parity']['max_rel_err'])
"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc -o kt -- python3 bench.py --config conformer --steps 8 --warmup 3 \
  --no-cpu-baseline --no-parity --no-roofline > $O/conf.log 2>&1 || { tail -20 $O/conf.log; exit 1; }
python3 tools/step_breakdown.py $O/tc 8 40 --gemm > $O/conformer_replay_step.txt 2>&1; head -3 $O/conformer_replay_step.txt
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
