# Round-3 measurement baseline: per-shape GEMM PMC census (+ attention counters from the same passes),
# the bench line, and a rocprofv3 kernel-trace summary of a bench run.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03g; mkdir -p $O
bash tools/cmd_census_pmc.sh r03g/census base > $O/census.out 2>&1; echo "census rc=$?"; head -45 $O/census/census_base.txt
for k in 3 4; do db=$(find $O/census/p$k -name "*.db" | head -1); [ -n "$db" ] && python tools/pmc_summary.py $db attn16 >> $O/attn_pmc.txt 2>&1; done
cat $O/attn_pmc.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; r=$?; echo "bench rc=$r"; tail -1 $O/bench.json
case $r in 0) ;; *) tail -20 $O/bench.err; exit $r;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-parity --no-conformer > $O/prof.log 2>&1; echo "prof rc=$?"
python tools/prof_summary.py $O/prof 6 40 > $O/prof_summary.txt 2>&1; head -50 $O/prof_summary.txt
