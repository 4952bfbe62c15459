set -u
# round-5 measurement set: vendor GEMM yardstick, per-replayed-step kernel summaries of both bench
# configs, and the per-shape GEMM + attention PMC census of the base step (HEAD)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05c}; mkdir -p $O
timeout -k 10 300 python3 tools/gemm_vs_blas.py > $O/gemm_vs_blas.txt 2>&1 || { tail $O/gemm_vs_blas.txt; exit 1; }
tail -3 $O/gemm_vs_blas.txt
for C in base conformer; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$C -o kt -- python3 bench.py --config $C --steps 10 --warmup 3 \
    --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/bench_$C.json 2> $O/bench_$C.err \
    || { tail -20 $O/bench_$C.err; exit 1; }
  MS=$(python3 -c "import json,sys; print(json.loads(open('$O/bench_$C.json').read().strip().splitlines()[-1])['ms_per_step'])")
  python3 tools/replay_summary.py $O/t_$C 10 45 $MS > $O/replay_summary_$C.txt 2>&1; head -3 $O/replay_summary_$C.txt
  find $O/t_$C -name "*.db" -delete; find $O/t_$C -name "*trace.csv" -delete
done
# GRU "single-CU floor" (VERDICT r4 item 6): gru16 (one CU per direction x 16 rows) vs grumc (the same
# recurrence split over H/64 = 4 CUs exchanging h through L2) on the headline step
for G in 1 0; do
  B2P_GRU16=$G timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-conformer \
    --no-extra --no-roofline > $O/gru16_$G.json 2> $O/gru16_$G.err || { tail -5 $O/gru16_$G.err; exit 1; }
  echo "B2P_GRU16=$G $(python3 -c "import json; print(json.loads(open('$O/gru16_$G.json').read().strip().splitlines()[-1])['ms_per_step'])") ms/step"
done
B2P_GRU16=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_grumc -o kt -- python3 bench.py --steps 10 --warmup 3 \
  --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/bench_grumc.json 2> $O/bench_grumc.err \
  || { tail -20 $O/bench_grumc.err; exit 1; }
python3 tools/replay_summary.py $O/t_grumc 10 45 > $O/replay_summary_base_grumc.txt 2>&1; head -3 $O/replay_summary_base_grumc.txt
find $O/t_grumc -name "*.db" -delete; find $O/t_grumc -name "*trace.csv" -delete
bash tools/cmd_census_pmc.sh ${1:-r05c}/census base > $O/census.log 2>&1 || { tail $O/census.log; exit 1; }
echo DONE
