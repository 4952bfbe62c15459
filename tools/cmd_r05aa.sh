set -u
# Conformer conv module: BatchNorm writes the 16-bit pointwise-conv-2 operands (no fp32 output, no casts)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "batchnorm or conv_module or conformer" \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
for V in 0 1; do
  B2P_BN16=$V timeout -k 10 300 python3 bench.py --config conformer --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$V.json 2> $O/b_$V.err || { tail -5 $O/b_$V.err; exit 1; }
  echo "conformer BN16=$V $(python3 -c "import json; print(json.loads(open('$O/b_$V.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_layerdrop_gpu.py tests/test_dp_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/tests2.log 2>&1
rc=$?; tail -2 $O/tests2.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests2.log | head -20; exit $rc; }
echo DONE
