set -u
# step-time A/B of environment switches: bash tools/cmd_ab_env.sh <tag> "<ENV=..>" ["<ENV=..>" ...]
# (default first; each variant runs the base + nested Conformer bench without baseline / parity / roofline)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for V in "" "$@"; do
  i=$((i+1))
  env $V timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity --no-roofline > $O/ab$i.log 2>&1 || { echo "variant '$V' failed"; tail -5 $O/ab$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/ab$i.log') if l.startswith('{')][-1]); print(repr('$V' or 'default'), d['ms_per_step'], d['conformer_large']['ms_per_step'])"
done
