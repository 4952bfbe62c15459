set -u
# The N > 1 bench path on a one-GPU box: two ranks over gloo sharing the GPU, launched as the driver
# launches N > 1 (torch.distributed.run, 127.0.0.1); the driver's own N > 1 runs use RCCL, one rank per GPU.
# usage: bash tools/cmd_dp_rehearsal.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dp}; mkdir -p $O
B2P_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-roofline > $O/dp2.log 2>&1 \
  || { tail -30 $O/dp2.log; exit 1; }
grep '^{' $O/dp2.log | tail -1 | cut -c1-600
