set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -s -k "split_bf16 or epilogue or nt_nn_tn" --timeout 120 --timeout-method thread > $O/gemm.log 2>&1
rc=$?; grep -E "bf16x3|passed|failed|Error" $O/gemm.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_configs34_gpu.py -x -q -s -k "bf16 and ft" --timeout 280 --timeout-method thread > $O/ft.log 2>&1
rc=$?; grep -E "rel \[|passed|failed" $O/ft.log | tail -4; [ $rc -ne 0 ] && exit $rc
for X in 0 1; do
B2P_X3_SPLIT=$X timeout -k 10 400 python3 -c "
import sys, json; sys.argv=['bench.py','--steps','10','--warmup','3']
import bench, torch
from wav2vec2forbrain_amd import build_lib; build_lib.ensure_built()
import argparse
from wav2vec2forbrain_amd import functional as Fn
Fn.set_precision('bf16')
args = argparse.Namespace(steps=10, warmup=3, bs=32, seq=1024, evaluator=False, no_roofline=False, graph=None)
r = bench.timed_run('conformer_ft', args, 1, 0, 'cuda:0', True)
print('X3_SPLIT=$X', r['precision'], round(r['dt']/r['steps']*1e3, 2), 'ms/step', 'gemm', [round(x,2) for x in r['gemm'][:2]])
" > $O/ft_$X.txt 2>&1 || { tail $O/ft_$X.txt; exit 1; }
tail -1 $O/ft_$X.txt
done
