cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 900 python -u tools/nested_probe.py conf_twice base_graph > $O/nested.txt 2>&1; r=$?; echo "rc=$r"
grep -E "base|conformer|==" $O/nested.txt
exit $r
