set -u
# mid-round checkpoint at HEAD: the driver's GPU commands (rehearsal), then per-replayed-step kernel
# summaries of both bench configs and the GEMM + attention PMC census of the base step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r05s}; O=gpurun_out/$T; mkdir -p $O
bash tools/cmd_rehearsal.sh $T || exit 1
for C in base conformer; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$C -o kt -- python3 bench.py --config $C --steps 10 --warmup 3 \
    --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/tbench_$C.json 2> $O/tbench_$C.err \
    || { tail -20 $O/tbench_$C.err; exit 1; }
  MS=$(python3 -c "import json,sys; print(json.loads(open('$O/tbench_$C.json').read().strip().splitlines()[-1])['ms_per_step'])")
  python3 tools/replay_summary.py $O/t_$C 10 45 $MS > $O/replay_summary_$C.txt 2>&1; head -3 $O/replay_summary_$C.txt
  find $O/t_$C -name "*.db" -delete; find $O/t_$C -name "*trace.csv" -delete
done
bash tools/cmd_census_pmc.sh $T/census base > $O/census.log 2>&1 || { tail $O/census.log; exit 1; }
echo DONE
