set -u
# A/B on one box: LayerDrop select with / without the fp16 copy (B2P_LD_SELECT_H)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05at; mkdir -p $O
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run base_h1 base && run base_h0 base B2P_LD_SELECT_H=0 && run base_h1b base && run base_h0b base B2P_LD_SELECT_H=0 && \
run large_h1 large && run large_h0 large B2P_LD_SELECT_H=0 || exit 1
