set -u
# GEMM HBM traffic of the current tree (base and Conformer bench commands): separate PMC passes
# FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md HBM section: FETCH x2 gfx950 correction in tools/traffic.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n; mkdir -p $O
for C in base conformer; do
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/${C}_fetch -o pmc -- python3 bench.py --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/${C}_fetch.log 2>&1 \
    || { tail -20 $O/${C}_fetch.log; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/${C}_write -o pmc -- python3 bench.py --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/${C}_write.log 2>&1 \
    || { tail -20 $O/${C}_write.log; exit 1; }
  python tools/traffic.py $(find $O/${C}_fetch -name "*.db" | head -1) $(find $O/${C}_write -name "*.db" | head -1) $O/gemm_traffic_$C.json
  cat $O/gemm_traffic_$C.json | head -c 600; echo
done
