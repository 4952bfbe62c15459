#!/bin/bash
# GPU check: selected parity tests (-k filter, optional) + bench line + rocprof kernel stats of the bench.
# usage: tools/gpu_check.sh <outdir> [pytest -k expr] [bench args...]
set -u
export TMPDIR=/tmp
O=gpurun_out/$1; K=${2:-}; shift; shift || true
mkdir -p $O
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1; rc=$?
  tail -8 $O/pytest.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || stop pytest $rc
  [ $rc -eq 0 ] || stop pytest-failed $rc
fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $O/bench.json 2>&1 || stop bench $?
tail -1 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" > $O/prof.log 2>&1 || stop prof $?
python tools/prof_summary.py $O/prof 6 30 > $O/prof_summary.txt 2>&1
head -20 $O/prof_summary.txt
echo DONE
