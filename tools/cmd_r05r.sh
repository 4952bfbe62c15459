set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > $O/attn_tests.log 2>&1
rc=$?; tail -2 $O/attn_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/attn_tests.log | head; exit $rc; }
for V in 0 1; do B2P_ATTN_T1=$V timeout -k 10 120 python3 tools/attn_bench.py > $O/attn_bench_$V.txt 2>&1 || exit 1; echo "T1=$V"; cat $O/attn_bench_$V.txt; done
for V in 0 1; do
  B2P_ATTN_T1=$V timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-conformer \
    --no-extra --no-roofline > $O/b_$V.json 2> $O/b_$V.err || { tail -5 $O/b_$V.err; exit 1; }
  echo "base ATTN_T1=$V $(python3 -c "import json; print(json.loads(open('$O/b_$V.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
