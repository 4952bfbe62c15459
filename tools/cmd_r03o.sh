cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 400 python -u tools/graph_probe.py conformer > $O/gp.txt 2>&1; echo "gp rc=$?"; grep graph $O/gp.txt
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 python -u tools/graph_probe.py conformer > $O/gp_nopc.txt 2>&1; echo "gp nopc rc=$?"; grep graph $O/gp_nopc.txt
timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA -d $O/a1 -o pmc -- python3 tools/attn_bench.py > $O/a1.log 2>&1; echo "pmc1 rc=$?"
timeout -k 10 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/a2 -o pmc -- python3 tools/attn_bench.py > $O/a2.log 2>&1; echo "pmc2 rc=$?"
for k in a1 a2; do db=$(find $O/$k -name "*.db" | head -1); [ -n "$db" ] && python3 tools/pmc_summary.py $db attn16 >> $O/attn_pmc.txt 2>&1; done
cat $O/attn_pmc.txt | head -150
find $O -name "*.db" -delete
