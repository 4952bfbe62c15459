set -u
# frozen weight gradients flushed every N encoder blocks, the batched launches spanning only the flushed
# layers' slots; batched weight-gradient tests first
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wgrad_batch_gpu.py tests/test_layerdrop_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B2P_WGRAD_FLUSH=block timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wgrad_batch_gpu.py > $O/tests_block.log 2>&1 || { tail -30 $O/tests_block.log; exit 1; }
tail -1 $O/tests_block.log
bash tools/cmd_ab_env.sh r06s_flush "B2P_WGRAD_FLUSH=block" "B2P_WGRAD_FLUSH=block:4" "B2P_WGRAD_FLUSH=block:8" || exit 1
