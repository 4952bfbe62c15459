set -u
# A/B of split-K for the deferred frozen-weight gradient GEMMs (B2P_DEFER_SPLIT)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/split; mkdir -p $O
for v in 1 0; do
  B2P_DEFER_SPLIT=$v timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --no-parity --steps 10 --warmup 3 > $O/c$v.json 2> $O/c$v.err || { tail -5 $O/c$v.err; exit 1; }
  echo "== conformer split=$v"; tail -1 $O/c$v.json | cut -c1-200
  B2P_DEFER_SPLIT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > $O/b$v.json 2> $O/b$v.err || { tail -5 $O/b$v.err; exit 1; }
  echo "== base split=$v"; tail -1 $O/b$v.json | cut -c1-200
done
B2P_DEFER_SPLIT=0 B2P_SIDE_STREAMS=2 timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --no-parity --steps 10 --warmup 3 > $O/c0s2.json 2> $O/c0s2.err || { tail -5 $O/c0s2.err; exit 1; }
echo "== conformer split=0 sides=2"; tail -1 $O/c0s2.json | cut -c1-200
