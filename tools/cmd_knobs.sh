set -u
# in-step A/B of GEMM tile knobs on the final tree
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs; mkdir -p $O
run() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; echo "$n $(grep '^{' $O/$n.json | cut -c80-140)"; }
run base_default B2P_X=0
run base_k64auto B2P_GEMM16_K64=-1
run base_k64 B2P_GEMM16_K64=1
run base_pp0 B2P_GEMM16_PP=0
run base_default2 B2P_X=0
