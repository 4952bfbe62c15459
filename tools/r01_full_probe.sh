#!/bin/bash
# full GPU parity suite + 1-GPU bench line (+ optional rocprof kernel stats of the bench)
set -u
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || stop pytest $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2>&1 || stop bench $?
tail -2 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || stop prof $?
echo DONE
