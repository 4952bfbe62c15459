cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03t; mkdir -p $O
for K in -1 0; do
B2P_GEMM16_K64=$K timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/k64_$K.json 2> $O/k64_$K.err; r=$?; echo "k64=$K rc=$r"
[ $r -eq 0 ] || { tail -5 $O/k64_$K.err; exit $r; }
tail -1 $O/k64_$K.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['conformer_large']; print('base', d['ms_per_step'], d['roofline']['frac'], 'conformer', c['ms_per_step'], c['roofline']['frac'])"
done
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_model_gpu.py -k "golden or gemm" > $O/pytest.log 2>&1; echo "tests rc=$?"; tail -3 $O/pytest.log
