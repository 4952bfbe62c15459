set -u
# narrow ping-pong GEMM: GEMM / model tests, the A/B against the 128 x 128 kernel, base / Conformer bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_layerdrop_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | tail; exit $rc; }
timeout -k 10 300 python3 -u tools/gemm_pn_ab.py 5 > $O/pn_ab.txt 2>&1 || { tail -5 $O/pn_ab.txt; exit 1; }; grep -v amdgpu $O/pn_ab.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('base', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['max_rel_err'])
c=d['conformer_large']; print('conformer', c['value'], c['ms_per_step'], c['roofline']['frac'], c['parity']['max_rel_err'])
"
