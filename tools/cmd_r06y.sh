set -u
# 64 x 64 tiles for under-filled narrow-N fp32-operand GEMMs (the lm_head): GEMM / model / trajectory tests, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_configs34_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/cmd_ab_env.sh r06y_step "B2P_LIB_PATH=probe_bin/libb2p_hip_prev.so" || exit 1
