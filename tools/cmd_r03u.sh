cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py "tests/test_model_gpu.py::test_step_matches_reference_golden" > $O/pytest.log 2>&1; r=$?; echo "tests rc=$r"; tail -3 $O/pytest.log
case $r in 124|137|134|139) exit $r;; esac
for P in 1 0; do
B2P_LN_PREFETCH=$P timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $O/pf$P.json 2> $O/pf$P.err; r=$?; echo "ln_prefetch=$P rc=$r"
[ $r -eq 0 ] || { tail -5 $O/pf$P.err; exit $r; }
tail -1 $O/pf$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['conformer_large']; print('base', d['ms_per_step'], d['roofline']['frac'], 'conformer', c['ms_per_step'], c['roofline']['frac'])"
done
