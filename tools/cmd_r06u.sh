set -u
# 16-byte conv weight permutation and activation-backward kernels: exactness tests, GEMM / kernel / model
# tests, step A/B against the library before round 6's element-pass changes (probe_bin/libb2p_hip_prev.so)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/cmd_ab_env.sh r06u_step "B2P_LIB_PATH=probe_bin/libb2p_hip_prev.so" || exit 1
