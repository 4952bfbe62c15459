#!/bin/bash
# Round profile: full bench line (with cpu_baseline), rocprofv3 kernel stats of the bench, and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) for the GEMM family's HBM traffic. Outputs stay under
# gpurun_out/<tag>/ (databases deleted after use: gpurun copies back at most 64 MiB); copy what is to be
# kept into profiles/ afterwards. usage: tools/round_profile.sh <tag>
set -u
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || stop smoke $?
grep smoke: $O/smoke.txt
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-conformer > $O/pmc_fetch.log 2>&1 || stop fetch $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-conformer > $O/pmc_write.log 2>&1 || stop write $?
python tools/traffic.py $(find $O/pmc_fetch -name "*.db" | head -1) $(find $O/pmc_write -name "*.db" | head -1) $O/gemm_traffic.json || stop traffic $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_c -o pmc -- python3 bench.py --config conformer --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_fetch_c.log 2>&1 || stop fetch_c $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_c -o pmc -- python3 bench.py --config conformer --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_write_c.log 2>&1 || stop write_c $?
python tools/traffic.py $(find $O/pmc_fetch_c -name "*.db" | head -1) $(find $O/pmc_write_c -name "*.db" | head -1) $O/gemm_traffic_conformer.json || stop traffic_c $?
find $O -name "*.db" -delete
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-parity --no-conformer > $O/prof.log 2>&1 || stop prof $?
python tools/prof_summary.py $O/prof 6 40 > $O/prof_summary.txt 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c -o run -- python3 bench.py --config conformer --steps 4 --warmup 2 --no-cpu-baseline --no-parity > $O/prof_c.log 2>&1 || stop prof_c $?
python tools/prof_summary.py $O/prof_c 6 40 > $O/prof_summary_conformer.txt 2>&1
find $O -name "*.db" -delete; find $O -name "*kernel_trace.csv" -delete
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || stop bench $?
tail -1 $O/bench.json
echo DONE
