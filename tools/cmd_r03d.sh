cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 900 python -u tools/trainer_capture_probe.py > $O/probe.txt 2>&1
echo "probe rc=$?"; grep -E "==|OK|step|Fatal|Error" $O/probe.txt | head -40
timeout -k 10 600 python -u -m pytest -m gpu -v --tb=short --timeout 300 --timeout-method thread tests/test_decode_gpu.py::test_cer_overflow_row_scored_on_host tests/test_dp_gpu.py::test_dp_replayed_trainer_steps_equal_global_batch_steps "tests/test_kernels_gpu.py::test_fused_attention_bf16_vs_fp32_core" tests/test_layerdrop_gpu.py::test_captured_layerdrop_adam_leaves_dropped_layers tests/test_model_gpu.py::test_step_graph_replay_matches_eager "tests/test_model_gpu.py::test_step_matches_reference_golden[fp32-conformer_large_ft_bs8]" > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Fatal|^E " $O/pytest.log | tail -40
exit $rc
