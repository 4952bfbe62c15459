cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 400 python -u tools/nested_probe.py conf_twice > $O/nested_reset.txt 2>&1; echo "reset rc=$?"; grep -E "conformer" $O/nested_reset.txt
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/nested_probe.py conf_twice > $O/nested_q8.txt 2>&1; echo "q8 rc=$?"; grep -E "conformer" $O/nested_q8.txt
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 400 python -u tools/nested_probe.py conf_twice > $O/nested_fgq4.txt 2>&1; echo "fgq4 rc=$?"; grep -E "conformer" $O/nested_fgq4.txt
timeout -k 10 300 python bench.py --config conformer --graph 0 --steps 6 --warmup 2 --no-cpu-baseline --no-parity --no-roofline > $O/conf_eager.json 2>$O/conf_eager.err; echo "conf eager rc=$?"; tail -1 $O/conf_eager.json | cut -c1-200
timeout -k 10 200 python -u tools/attn_bench.py > $O/attn.txt 2>&1; echo "attn rc=$?"; grep attn16 $O/attn.txt
