set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z3; mkdir -p $O
timeout -k 10 300 python3 tools/blaslt_count.py conformer > $O/count_conf.txt 2>&1 || { tail -20 $O/count_conf.txt; exit 1; }
grep -v amdgpu.ids $O/count_conf.txt | head -60
for V in 0 1; do
  B2P_BLASLT=$V timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc$V -o kt -- python3 bench.py --config conformer --steps 6 --warmup 3 --no-cpu-baseline \
    --no-parity --no-roofline --no-conformer --no-extra > $O/conf$V.log 2>&1 || { tail -20 $O/conf$V.log; exit 1; }
  python3 tools/step_breakdown.py $O/tc$V 6 60 > $O/conf_replay_step_$V.txt 2>&1; head -1 $O/conf_replay_step_$V.txt
  find $O/tc$V -name "*.db" -delete; find $O/tc$V -name "*.csv" -delete
done
