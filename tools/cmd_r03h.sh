cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v -s --tb=short --timeout 300 --timeout-method thread "tests/test_kernels_gpu.py::test_fused_attention_bf16_vs_fp32_core" tests/test_configs34_gpu.py "tests/test_model_gpu.py::test_step_matches_reference_golden" > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Fatal|^E |rel \[|worst" $O/pytest.log | tail -70
case $rc in 124|137|134|139) echo "stop after pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -u tools/fixture_err.py conformer_large_b2 large960_bs32 conformer_large_ft_bs8 > $O/fixture_err.txt 2>&1; echo "fixture_err rc=$?"
grep -E "fp32\[-\]|all-fp32" $O/fixture_err.txt
for T in 0 1; do
  B2P_GEMM16_TALL=$T timeout -k 10 120 python -u tools/gemm_ab.py > $O/gemm_ab_t$T.txt 2>&1 || { r=$?; echo "gemm_ab rc=$r"; tail -3 $O/gemm_ab_t$T.txt; exit $r; }
  grep -v amdgpu.ids $O/gemm_ab_t$T.txt
done
exit $rc
