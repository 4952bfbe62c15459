set -u
# float4 BatchNorm input-gradient pass with the scalar form's rounding sequence: bitwise test, Conformer
# model / trajectory tests, step A/B against B2P_BN_DX4=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_configs34_gpu.py -k "conv_module or conformer or conf" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/cmd_ab_env.sh r06aa_step "B2P_BN_DX4=0" || exit 1
