set -u
# per-shape GEMM PMC census of the base step at the end of round 5 (hbm/alg per launch kind)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/cmd_census_pmc.sh r05ax base > gpurun_out/r05ax_census.log 2>&1 || { tail -20 gpurun_out/r05ax_census.log; exit 1; }
head -30 gpurun_out/r05ax/census_base.txt | cut -c1-110
