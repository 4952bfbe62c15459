set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05g; mkdir -p $O
B2P_WGRAD_DEBUG=1 timeout -k 10 250 python3 bench.py --config conformer --steps 2 --warmup 2 --no-cpu-baseline --no-parity --no-roofline > $O/dbg.txt 2>&1 || { tail $O/dbg.txt; exit 1; }
grep wgrad $O/dbg.txt | sort | uniq -c | head -30
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_layerdrop_gpu.py tests/test_trainer_gpu.py tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for C in conformer base; do for W in 0 1; do
  B2P_WGRAD_BATCH=$W timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_${C}_$W.json 2> $O/b_${C}_$W.err || { tail -5 $O/b_${C}_$W.err; exit 1; }
  echo "$C WGRAD_BATCH=$W $(python3 -c "import json; print(json.loads(open('$O/b_${C}_$W.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done; done
