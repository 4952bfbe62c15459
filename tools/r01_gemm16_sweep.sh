#!/bin/bash
# bf16 GEMM: parity tests, then the shape sweep for each (KT, stages) variant.
set -u
export TMPDIR=/tmp
O=gpurun_out/sweep16
mkdir -p $O
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > $O/pytest_gemm.log 2>&1; rc=$?
tail -15 $O/pytest_gemm.log
[ $rc -eq 0 ] || stop pytest $rc
for cfg in 64,2 64,3 32,2 32,3 32,4; do
  B2P_GEMM16=$cfg timeout -k 10 300 python tools/bench_gemm.py b16 > $O/gemm_b16_$cfg.jsonl 2>&1 || stop gemm_$cfg $?
done
for cfg in 64,2 64,3 32,2 32,3 32,4; do echo "== $cfg"; cat $O/gemm_b16_$cfg.jsonl | grep shape; done
echo DONE
