set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/grumc; mkdir -p $O
timeout -k 10 150 python tools/grumc_debug.py > $O/debug.txt 2>&1 || { tail -20 $O/debug.txt; exit 1; }
grep "vs fp32" $O/debug.txt
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gru" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 120 python tools/gru512_bench.py > $O/mc.txt 2>&1 || { tail -20 $O/mc.txt; exit 1; }
echo "multi-CU:"; tail -1 $O/mc.txt
timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --no-parity --no-roofline > $O/conf.json 2> $O/conf.err || { tail -5 $O/conf.err; exit 1; }
python -c "import json; d=json.loads(open('$O/conf.json').read().strip().splitlines()[-1]); print('conformer ms/step', d['ms_per_step'])"
