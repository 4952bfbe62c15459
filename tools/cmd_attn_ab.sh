# attention variant A/B (kernel microbenchmark): default library vs B2P_LIB_PATH=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/attn_ab; mkdir -p $O
timeout -k 10 120 python -u tools/attn_bench.py > $O/default.txt 2>&1; echo "default rc=$?"; grep attn16 $O/default.txt
B2P_LIB_PATH=$1 timeout -k 10 120 python -u tools/attn_bench.py > $O/variant.txt 2>&1; echo "variant rc=$?"; grep attn16 $O/variant.txt
