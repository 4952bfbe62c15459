set -u
# LayerDrop select writing the fp16 copy too (post-LN forward_f16 layers read it uncast): LayerDrop /
# trainer / model tests, step times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05as; mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_layerdrop_gpu.py tests/test_trainer_gpu.py \
  tests/test_model_gpu.py tests/test_configs34_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run base base && run base_b base && run large large || exit 1
