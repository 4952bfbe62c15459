set -u
# Round profile r01f, Conformer-large config: kernel stats of the bench command, then the bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r01f_conf
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config conformer --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 \
  || { tail -20 $O/prof.log; exit 1; }
python tools/prof_summary.py $O/prof 6 40 > $O/prof_summary.txt 2>&1
timeout -k 10 500 python bench.py --config conformer --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
