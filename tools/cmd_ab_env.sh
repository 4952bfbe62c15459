# Step-level A/B of environment switches: bash tools/cmd_ab_env.sh <tag> "<VAR=a>" "<VAR=b>" ...
# (bench.py without CPU baseline / parity: base line + nested Conformer record per setting)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift; mkdir -p $O
for V in "$@"; do
  F=$(echo "$V" | tr '/=' '__')
  env $V timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$O/$F.json" 2> "$O/$F.err"; r=$?
  echo "$V rc=$r"; [ $r -eq 0 ] || { tail -5 "$O/$F.err"; exit $r; }
  tail -1 "$O/$F.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['conformer_large']; print('  base', d['ms_per_step'], d['roofline']['frac'], 'conformer', c['ms_per_step'], c['roofline']['frac'])"
done
