set -u
# frozen weight-gradient batch groups keyed by (rows, numel) per parameter (B2P_WGRAD_MERGE): tests, A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aw; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wgrad_batch_gpu.py tests/test_model_gpu.py \
  tests/test_trainer_gpu.py tests/test_layerdrop_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run conf_m1 conformer && run conf_m0 conformer B2P_WGRAD_MERGE=0 && run conf_m1b conformer && run conf_m0b conformer B2P_WGRAD_MERGE=0 && \
run base_m1 base || exit 1
