set -u
# GEMM tile-order / stage-count sweep on the encoder shapes (bf16 operands)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i_order; mkdir -p $O
for v in "G0 0 0" "G4 4 0" "G8 8 0" "G16 16 0" "S4 0 1" "S4G8 8 1"; do
  set -- $v
  B2P_GEMM16_GROUP=$2 B2P_GEMM16_S4=$3 timeout -k 10 120 python tools/bench_gemm.py b16 > $O/$1.jsonl 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  echo "== $1"; cat $O/$1.jsonl
done
