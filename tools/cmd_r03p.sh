cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 400 python -u tools/nested_probe.py conf_twice_nodefer > $O/n1.txt 2>&1; echo "nodefer rc=$?"; grep -E "conformer" $O/n1.txt
B2P_GRAPH_PRIORITY=0 timeout -k 10 400 python -u tools/nested_probe.py conf_twice > $O/n2.txt 2>&1; echo "prio0 rc=$?"; grep -E "conformer" $O/n2.txt
