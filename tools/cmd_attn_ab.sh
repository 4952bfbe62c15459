# attention variant A/B: kernel microbenchmark and the step, default library vs B2P_LIB_PATH=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/attn_ab; mkdir -p $O
V=$1
timeout -k 10 120 python -u tools/attn_bench.py > $O/default.txt 2>&1; echo "default rc=$?"; grep attn16 $O/default.txt
B2P_LIB_PATH=$V timeout -k 10 120 python -u tools/attn_bench.py > $O/variant.txt 2>&1; echo "variant rc=$?"; grep attn16 $O/variant.txt
B2P_LIB_PATH=$V timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread "tests/test_kernels_gpu.py::test_fused_attention_bf16_vs_fp32_core" > $O/pytest.log 2>&1; echo "variant tests rc=$?"; tail -2 $O/pytest.log
bash tools/cmd_ab_env.sh attn_ab_step "B2P_LIB_PATH=" "B2P_LIB_PATH=$V"
