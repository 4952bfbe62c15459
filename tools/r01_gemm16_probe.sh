#!/bin/bash
# GPU probe for the bf16-operand GEMM: parity tests, shape sweep, PMC on FFN1 (NT/NN/TN).
set -u
export TMPDIR=/tmp
O=gpurun_out/probe16
mkdir -p $O
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > $O/pytest_gemm.log 2>&1; rc=$?
tail -15 $O/pytest_gemm.log
[ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python tools/bench_gemm.py b16 > $O/gemm_b16.jsonl 2>&1 || stop gemm_b16 $?
cat $O/gemm_b16.jsonl
for kind in nt nn tn; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/pmc_sq_$kind -o pmc -- python3 tools/gemm_one.py $kind 7968 3072 768 20 b16 > $O/pmc_sq_$kind.log 2>&1 || stop pmc_$kind $?
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_nt -o pmc -- python3 tools/gemm_one.py nt 7968 3072 768 20 b16 > $O/pmc_fetch_nt.log 2>&1 || stop fetch $?
echo DONE
