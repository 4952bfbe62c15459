cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03q; mkdir -p $O
for P in 0 1; do
B2P_GRAPH_PRIORITY=$P timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/prio$P.json 2> $O/prio$P.err; r=$?; echo "prio=$P rc=$r"
[ $r -eq 0 ] || { tail -5 $O/prio$P.err; exit $r; }
tail -1 $O/prio$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['conformer_large']; print('base', d['ms_per_step'], d['roofline']['frac'], 'conformer', c['ms_per_step'], c['roofline']['frac'])"
done
