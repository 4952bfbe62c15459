cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v -s --tb=short --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_layerdrop_gpu.py tests/test_model_gpu.py::test_step_graph_replay_matches_eager tests/test_configs34_gpu.py "tests/test_model_gpu.py::test_step_matches_reference_golden" > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Fatal|^E |rel \[|worst" $O/pytest.log | tail -60
case $rc in 124|137|134|139) echo "stop after pytest rc=$rc"; exit $rc;; esac
for G in 0 -1; do for T in 0 1; do
  B2P_GEMM16_GROUP=$G B2P_GEMM16_TALL=$T timeout -k 10 120 python -u tools/gemm_ab.py > $O/gemm_ab_g${G}_t$T.txt 2>&1 || { r=$?; echo "gemm_ab rc=$r"; tail -3 $O/gemm_ab_g${G}_t$T.txt; exit $r; }
  cat $O/gemm_ab_g${G}_t$T.txt | grep -v amdgpu.ids
done; done
exit $rc
