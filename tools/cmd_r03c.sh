cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u tools/fixture_err.py conformer_large_b2 large960_bs32 conformer_large_ft_bs8 > $O/fixture_err.txt 2>&1 || { echo "fixture_err rc=$?"; tail -5 $O/fixture_err.txt; exit 1; }
cat $O/fixture_err.txt
timeout -k 10 600 python -u -m pytest -m gpu -v --tb=short --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_decode_gpu.py::test_cer_overflow_row_scored_on_host tests/test_dp_gpu.py::test_dp_replayed_trainer_steps_equal_global_batch_steps "tests/test_kernels_gpu.py::test_fused_attention_bf16_vs_fp32_core" tests/test_layerdrop_gpu.py::test_captured_layerdrop_adam_leaves_dropped_layers tests/test_model_gpu.py::test_step_graph_replay_matches_eager "tests/test_model_gpu.py::test_step_matches_reference_golden[fp32-conformer_large_ft_bs8]" > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Fatal" $O/pytest.log | tail -40
exit $rc
