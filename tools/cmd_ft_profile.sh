set -u
# kernel statistics of the configs[4] per-GPU step under the per-role bf16x3 policy (tools/ft_policy_ab.py:
# 3 eager warm-up steps, the capture, 10 replays, the fixture trajectory). usage: bash tools/cmd_ft_profile.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ft_prof}; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/ft_policy_ab.py "wgrad,dgrad2b" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof 14 30 > $O/prof_summary_ft.txt 2>&1
head -32 $O/prof_summary_ft.txt
find $O/prof -name "*.db" -delete; find $O/prof -name "*kernel_trace.csv" -delete
