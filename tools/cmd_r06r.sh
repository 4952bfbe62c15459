set -u
# Clean GEMM traffic at HEAD: side-stream work serialised into the main stream (B2P_SERIAL_SIDE=1), so the
# per-dispatch PMC counters see one kernel at a time. Per-shape census of the base step (4 passes), then
# FETCH_SIZE / WRITE_SIZE passes over eager steps of configs[1]..[4] for bench.py's roofline.traffic.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export B2P_SERIAL_SIDE=1
O=gpurun_out/r06r; mkdir -p $O
bash tools/cmd_census_pmc.sh r06r_census base > $O/census_head.txt 2>&1 || { tail -20 $O/census_head.txt; exit 1; }
head -30 $O/census_head.txt
for K in base conformer large conformer_ft; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/f_$K -o pmc -- python3 tools/traffic_run.py $K > $O/f_$K.log 2>&1 || { echo "fetch $K failed"; tail -5 $O/f_$K.log; find $O -name "*.db" -delete; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/w_$K -o pmc -- python3 tools/traffic_run.py $K > $O/w_$K.log 2>&1 || { echo "write $K failed"; tail -5 $O/w_$K.log; find $O -name "*.db" -delete; exit 1; }
  S=$([ $K = base ] && echo "" || echo "_$K")
  python3 tools/traffic.py $(find $O/f_$K -name "*.db" | head -1) $(find $O/w_$K -name "*.db" | head -1) $O/r06r_gemm_traffic$S.json || exit 1
  find $O -name "*.db" -delete
done
