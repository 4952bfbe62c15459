cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 1100 python -u tools/nested_probe.py > $O/nested.txt 2>&1; r=$?; echo "rc=$r"
grep -E "base|conformer|==" $O/nested.txt
exit $r
