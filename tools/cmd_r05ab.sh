set -u
# where the remaining 16-bit cast passes sit in a replayed Conformer step (neighbours of every cast kernel)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_conf -o kt -- python3 bench.py --config conformer --steps 3 --warmup 2 \
  --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/tconf.json 2> $O/tconf.err || { tail -20 $O/tconf.err; exit 1; }
python3 tools/step_dump.py $O/t_conf "cast16_2d,cast_bf16,cast16_tail,pad_rows16,colsum_fold_v" 1 > $O/conf_cast_dump.txt 2>&1; grep -c "^>" $O/conf_cast_dump.txt
python3 tools/replay_summary.py $O/t_conf 2 70 > $O/conf_summary.txt 2>&1; head -3 $O/conf_summary.txt
find $O/t_conf -name "*.db" -delete; find $O/t_conf -name "*trace.csv" -delete
