set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ldab; mkdir -p $O
for v in "cur:" "ld0:B2P_DIAG_LAYERDROP=0" "old:B2P_GRAPH_LAYERDROP=0"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(python -c "import json,sys; d=json.load(open('$O/$n.json')); print(d['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-parity > $O/prof.log 2>&1 || exit 1
python tools/timeline.py $O/prof adam 1 > $O/timeline.txt 2>&1
head -60 $O/timeline.txt
