set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for C in base conformer; do
  O=gpurun_out/census_$C; mkdir -p $O
  CENSUS_CONFIG=$C timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/gemm_census.py run $O > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  python tools/gemm_census.py report $O > $O/report.txt 2>&1
  head -40 $O/report.txt
done
