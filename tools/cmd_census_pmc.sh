set -u
# Per-shape GEMM PMC table of one eager base step (tools/gemm_pmc_census.py): one rocprofv3 pass per
# counter set (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md HBM section).
# usage: bash tools/cmd_census_pmc.sh <tag> [base|conformer]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; C=${2:-base}; mkdir -p $O
export CENSUS_CONFIG=$C
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P -d $O/p$i -o pmc -- python3 tools/gemm_pmc_census.py run $O > $O/p$i.log 2>&1 \
    || { echo "pass $i ($P) failed"; tail -5 $O/p$i.log; find $O -name "*.db" -delete; exit 1; }
done
python3 tools/gemm_pmc_census.py report $O $(for k in 1 2 3 4; do find $O/p$k -name "*.db" | head -1; done) > $O/census_$C.txt 2>&1
head -40 $O/census_$C.txt
# the fused attention kernels' counters from the same passes, then drop the databases (gpurun copies
# back at most 64 MiB of gpurun_out/)
for k in 3 4; do db=$(find $O/p$k -name "*.db" | head -1); [ -n "$db" ] && python3 tools/pmc_summary.py $db attn16 >> $O/attn_pmc_$C.txt 2>&1; done
find $O -name "*.db" -delete
