set -u
# attention kernels at HEAD (tools/attn_bench.py, base shape B=32 T'=249 12 heads): times, and PMC in two
# passes (instruction mix / wait cycles; MFMA / LDS / bank conflicts), one rocprofv3 run per counter set
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05al; mkdir -p $O
timeout -k 10 120 python3 tools/attn_bench.py > $O/attn_bench.txt 2>&1 || { tail $O/attn_bench.txt; exit 1; }
cat $O/attn_bench.txt
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o pmc -- python3 tools/attn_bench.py > $O/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $O/p$i.log; find $O -name "*.db" -delete; exit 1; }
  db=$(find $O/p$i -name "*.db" | head -1); python3 tools/pmc_summary.py $db attn >> $O/attn_pmc.txt 2>&1
done
find $O -name "*.db" -delete
grep -c "" $O/attn_pmc.txt
