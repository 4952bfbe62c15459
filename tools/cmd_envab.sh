set -u
# A/B of environment settings on the bench: bash tools/cmd_envab.sh <config> "<NAME:ENV=..>" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/envab; mkdir -p $O
C=$1; shift
for v in "$@"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-parity --no-roofline > $O/$C-$n.json 2> $O/$C-$n.err || { tail -5 $O/$C-$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$C-$n.json').read().strip().splitlines()[-1]); print('$C $n', d['ms_per_step'])"
done
