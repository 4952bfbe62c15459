# Conformer step regression hunt: kernel stats of replayed Conformer steps, fp16 attention on / off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03i; mkdir -p $O
for A in 1 0; do
  B2P_ATTN_F16=$A timeout -k 10 400 python bench.py --config conformer --steps 6 --warmup 3 --no-cpu-baseline --no-parity --no-roofline > $O/bench_attnf16_$A.json 2> $O/bench_attnf16_$A.err; r=$?
  echo "attn_f16=$A rc=$r"; tail -1 $O/bench_attnf16_$A.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['step_mode'])"
  [ $r -eq 0 ] || { tail -5 $O/bench_attnf16_$A.err; exit $r; }
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config conformer --steps 4 --warmup 2 --no-cpu-baseline --no-parity --no-roofline > $O/prof.log 2>&1; echo "prof rc=$?"
python tools/prof_summary.py $O/prof 6 45 > $O/prof_summary.txt 2>&1; head -48 $O/prof_summary.txt
find $O/prof -name "*.db" -delete; find $O/prof -name "*.csv" -size +2M -delete; du -sh $O
