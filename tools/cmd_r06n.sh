set -u
# bf16x3 policy with per-role forms: trajectory tests (configs[1-4]) + the configs[4] bench record
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_configs34_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "sign-lost|passed|failed" $O/tests.log | tail -12
timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(gpus=1, steps=20, warmup=5, bs=32, seq=1024, no_cpu_baseline=True, no_parity=True, no_roofline=False,
                       no_conformer=True, no_extra=True, evaluator=False, graph=None, config='base')
r = bench.ft_record(a, 'cuda:0')
print(json.dumps(r))
" > $O/ft.log 2>&1 || { tail -30 $O/ft.log; exit 1; }
tail -1 $O/ft.log
