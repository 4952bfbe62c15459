set -u
# narrow ping-pong kernel for every k-contiguous launch (QKV N = 2304, pointwise-conv-1 N = 2048 ...)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o; mkdir -p $O
GEMM_AB_ONLY=7968x2304x768,7968x2048x1024 timeout -k 10 120 python3 tools/gemm_ab.py > $O/ab_default.log 2>&1 || { tail $O/ab_default.log; exit 1; }
B2P_GEMM16_PN=2 GEMM_AB_ONLY=7968x2304x768,7968x2048x1024 timeout -k 10 120 python3 tools/gemm_ab.py > $O/ab_pn2.log 2>&1 || { tail $O/ab_pn2.log; exit 1; }
cat $O/ab_default.log $O/ab_pn2.log | grep -v amdgpu.ids
bash tools/cmd_ab_env.sh r06o_step "B2P_GEMM16_PN=2" || exit 1
