#!/bin/bash
# GPU probe: parity suite, GEMM shape sweep for KB=32/64, PMC passes on the FFN1 shape, bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/probe
mkdir -p $O
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || stop pytest $rc
for kb in 32 64; do
  B2P_GEMM_KB=$kb timeout -k 10 300 python tools/bench_gemm.py > $O/gemm_kb$kb.jsonl 2>&1 || stop gemm$kb $?
done
for kb in 32 64; do
  B2P_GEMM_KB=$kb timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/pmc_sq_kb$kb -o pmc -- python3 tools/gemm_one.py nt 7968 3072 768 20 > $O/pmc_sq_kb$kb.log 2>&1 || stop pmc$kb $?
  B2P_GEMM_KB=$kb timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_kb$kb -o pmc -- python3 tools/gemm_one.py nt 7968 3072 768 20 > $O/pmc_fetch_kb$kb.log 2>&1 || stop fetch$kb $?
done
for kb in 32 64; do
  B2P_GEMM_KB=$kb timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_kb$kb.json 2>&1 || stop bench$kb $?
done
cat $O/bench_kb*.json
echo DONE
