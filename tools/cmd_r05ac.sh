set -u
# long-K split rule; frozen weight-gradient flush every N encoder blocks (A/B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ac; mkdir -p $O
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run base_longk0 base B2P_PP_SPLIT_LONG_K=1000000000 && run base_longk base B2P_PP_SPLIT_LONG_K=8192 && \
run base_every12 base B2P_WGRAD_FLUSH_EVERY=12 && \
run conf_longk0 conformer B2P_PP_SPLIT_LONG_K=1000000000 && run conf_longk conformer B2P_PP_SPLIT_LONG_K=8192 && \
run conf_every48 conformer B2P_WGRAD_FLUSH_EVERY=48 && run conf_every32 conformer B2P_WGRAD_FLUSH_EVERY=32 || exit 1
