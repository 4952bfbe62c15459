set -u
# N>1 rehearsal of bench.py on the one-GPU box: two gloo ranks sharing the GPU (the driver's N>1 runs use
# RCCL with one rank per GPU); checks the multi-rank step (graph replay + bucket exchange + Adam) runs.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dp2; mkdir -p $O
B2P_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
grep '^{' $O/bench2.json | cut -c1-400
