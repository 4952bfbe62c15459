cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/tr -o run -- python3 tools/nested_probe.py --one conf_twice > $O/probe.log 2>&1; echo "trace rc=$?"
grep -E "conformer" $O/probe.log
python tools/two_run_compare.py $O/tr 30 > $O/compare.txt 2>&1; cat $O/compare.txt
find $O/tr -name "*.db" -delete; find $O/tr -name "*.csv" -delete
