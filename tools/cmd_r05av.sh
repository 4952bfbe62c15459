set -u
# frozen Linear (lm_head) weight gradient on the side stream: tests, smoke, step-time A/B (B2P_LINEAR_WGRAD_DEFER)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05av; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_trainer_gpu.py \
  tests/test_layerdrop_gpu.py tests/test_wgrad_batch_gpu.py tests/test_dp_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run base_d1 base && run base_d0 base B2P_LINEAR_WGRAD_DEFER=0 && run base_d1b base && run base_d0b base B2P_LINEAR_WGRAD_DEFER=0 && \
run conf_d1 conformer && run conf_d0 conformer B2P_LINEAR_WGRAD_DEFER=0 || exit 1
