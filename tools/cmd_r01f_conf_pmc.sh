set -u
# GEMM HBM traffic of the Conformer-large bench command: two separate PMC passes (FETCH_SIZE, WRITE_SIZE).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r01f_conf
mkdir -p $O
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc -- python3 bench.py --config conformer --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 \
  || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc -- python3 bench.py --config conformer --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 \
  || { tail -20 $O/pmc_write.log; exit 1; }
python tools/traffic.py $(find $O/pmc_fetch -name "*.db" | head -1) $(find $O/pmc_write -name "*.db" | head -1) $O/gemm_traffic_conformer.json
