# nested Conformer record slowdown: which part of the base run before it matters
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python bench.py --steps 10 --warmup 3 "$@" > $O/$tag.json 2> $O/$tag.err; r=$?; echo "$tag rc=$r"; [ $r -eq 0 ] || { tail -5 $O/$tag.err; exit $r; }
  tail -1 $O/$tag.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['conformer_large']; print('base', d['ms_per_step'], 'conformer', c['ms_per_step'])"; }
run noroof_nocpu_nopar --no-roofline --no-cpu-baseline --no-parity
run roof_nocpu_nopar --no-cpu-baseline --no-parity
run noroof_cpu_nopar --no-roofline --no-parity
