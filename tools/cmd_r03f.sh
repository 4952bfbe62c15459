cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -v -s --tb=short --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_layerdrop_gpu.py tests/test_model_gpu.py::test_step_graph_replay_matches_eager tests/test_configs34_gpu.py "tests/test_model_gpu.py::test_step_matches_reference_golden" > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Fatal|^E |rel \[|worst" $O/pytest.log | tail -60
exit $rc
