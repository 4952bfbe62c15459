set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05f; mkdir -p $O
for C in conformer base; do for W in 0 1; do
  B2P_WGRAD_BATCH=$W timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_${C}_$W.json 2> $O/b_${C}_$W.err || { tail -5 $O/b_${C}_$W.err; exit 1; }
  echo "$C WGRAD_BATCH=$W $(python3 -c "import json; print(json.loads(open('$O/b_${C}_$W.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_c -o kt -- python3 bench.py --config conformer --steps 6 --warmup 3 \
    --no-cpu-baseline --no-parity --no-roofline > $O/bench_c.json 2> $O/bench_c.err || { tail -20 $O/bench_c.err; exit 1; }
python3 tools/replay_summary.py $O/t_c 6 50 > $O/replay_summary_conformer.txt 2>&1; head -30 $O/replay_summary_conformer.txt
find $O/t_c -name "*.db" -delete; find $O/t_c -name "*trace.csv" -delete
