set -u
# GEMM census (eager step, per-shape times) for both configs + replayed-step timeline of the base bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for C in base conformer; do
  O=gpurun_out/r02h_census_$C; mkdir -p $O
  CENSUS_CONFIG=$C timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/gemm_census.py run $O > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  python tools/gemm_census.py report $O > $O/report.txt 2>&1
  head -45 $O/report.txt
done
O=gpurun_out/r02h_prof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-parity > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O adam 1 > $O/timeline.txt 2>&1 || true
head -45 $O/timeline.txt
