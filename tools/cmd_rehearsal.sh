set -u
# round-end rehearsal: exactly the driver's GPU commands on this tree (pytest -m gpu, smoke(), the default
# bench line), each under its own time limit; usage: bash tools/cmd_rehearsal.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rehearsal}; mkdir -p $O
T0=$SECONDS
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; echo "pytest wall $((SECONDS - T0)) s"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | tail; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
T0=$SECONDS
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall $((SECONDS - T0)) s" | tee $O/bench_wall.txt
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('base', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['max_rel_err'], d.get('vs_cpu'))
c=d['conformer_large']; print('conformer', c['value'], c['ms_per_step'], c['roofline']['frac'], c['parity']['max_rel_err'])
print('evaluator', d['train_evaluator_record']['value'], 'fp32', d['fp32_mode']['value'])
l=d['large960']; print('large960', l['value'], l['ms_per_step'], l['parity']['max_rel_err'])
f=d['conformer_large_ft']; print('ft', f['value'], f['ms_per_step'], f['dtype'], f['parity']['max_rel_err'], 'policy_off', f['policy_off']['value'], f['policy_off']['parity']['max_rel_err'])
"
