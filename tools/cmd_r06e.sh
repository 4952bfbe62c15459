set -u
# quarter-scheduled operand DMA in the ping-pong GEMM: the GPU suite, the interleaved A/B, attention bench,
# base / Conformer bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | tail; exit $rc; }
timeout -k 10 300 python3 -u tools/gemm_qs_ab.py 5 > $O/qs_ab.txt 2>&1 || { tail -5 $O/qs_ab.txt; exit 1; }; grep -v amdgpu $O/qs_ab.txt
timeout -k 10 120 python3 tools/attn_bench.py > $O/attn_bench.txt 2>&1 || { tail -5 $O/attn_bench.txt; exit 1; }; grep attn16 $O/attn_bench.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('base', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['max_rel_err'])
c=d['conformer_large']; print('conformer', c['value'], c['ms_per_step'], c['roofline']['frac'], c['parity']['max_rel_err'])
"
