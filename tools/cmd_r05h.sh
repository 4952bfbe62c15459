set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wgrad_batch_gpu.py tests/test_model_gpu.py tests/test_configs34_gpu.py -v -s -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|rel \[|worst" $O/tests.log | tail -40; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for P in 0 1; do
  B2P_FFN_PRE16=$P timeout -k 10 300 python3 bench.py --config conformer --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-roofline > $O/b_$P.json 2> $O/b_$P.err || { tail -5 $O/b_$P.err; exit 1; }
  echo "conformer FFN_PRE16=$P $(python3 -c "import json; print(json.loads(open('$O/b_$P.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
