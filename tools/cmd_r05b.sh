set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_trainer_gpu.py -x -q -k "colsum or trainer" --timeout 120 --timeout-method thread > $O/kern.log 2>&1
rc=$?; tail -3 $O/kern.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_configs34_gpu.py -v -s --timeout 300 --timeout-method thread > $O/configs34.log 2>&1
rc=$?
grep -E "PASS|FAIL|rel \[|worst" $O/configs34.log | tail -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-conformer > $O/bench.json 2> $O/bench.err
rc2=$?
tail -5 $O/bench.err; tail -c 3000 $O/bench.json
exit $rc2
