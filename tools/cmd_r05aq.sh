set -u
# diagnostic: step time without the frozen weight-gradient launches (B2P_DIAG_SKIP_WGRAD=1): how much of
# the step's tail the side stream holds (not a valid bench setting)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aq; mkdir -p $O
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run base base && run base_nowgrad base B2P_DIAG_SKIP_WGRAD=1 && run conf conformer && run conf_nowgrad conformer B2P_DIAG_SKIP_WGRAD=1 || exit 1
