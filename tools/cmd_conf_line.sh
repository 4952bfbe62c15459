set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/conf_line; mkdir -p $O
timeout -k 10 400 python bench.py --config conformer --no-cpu-baseline --steps 10 --warmup 3 > $O/c.json 2> $O/c.err || { tail -5 $O/c.err; exit 1; }
grep '^{' $O/c.json
