set -u
# plain 16-bit GEMMs through hipBLASLt: parity tests (the library path against gemm16, the trajectories),
# then the step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_blaslt_gpu.py -x -q --timeout 200 --timeout-method thread > $O/blaslt_tests.log 2>&1
rc=$?; tail -2 $O/blaslt_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/blaslt_tests.log | head -20; exit $rc; }
for C in base conformer; do
  for V in 0 1; do
    B2P_BLASLT=$V timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
      --no-conformer --no-extra --no-roofline > $O/b_${C}_$V.json 2> $O/b_${C}_$V.err || { tail -5 $O/b_${C}_$V.err; exit 1; }
    echo "$C BLASLT=$V $(python3 -c "import json; print(json.loads(open('$O/b_${C}_$V.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_configs34_gpu.py tests/test_layerdrop_gpu.py tests/test_model_gpu.py tests/test_trainer_gpu.py -x -v -s \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E " rel \[|passed|failed" $O/tests.log | tail -14 | cut -c1-250; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
echo DONE
