set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z2; mkdir -p $O
for V in 0 1; do
  B2P_BLASLT=$V timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tb$V -o kt -- python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline \
    --no-parity --no-roofline --no-conformer --no-extra > $O/base$V.log 2>&1 || { tail -20 $O/base$V.log; exit 1; }
  python3 tools/step_breakdown.py $O/tb$V 8 60 > $O/base_replay_step_$V.txt 2>&1; head -2 $O/base_replay_step_$V.txt
  find $O/tb$V -name "*.db" -delete; find $O/tb$V -name "*.csv" -delete
done
