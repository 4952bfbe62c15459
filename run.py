"""Entry point — the reference's run.py (`experiment = get_experiment_from_args(); experiment.run()`)
on the MI355X build. Data-parallel: torchrun --nproc-per-node N run.py ... (one process per GPU,
RCCL; the Trainer all-reduces the gradient buckets)."""
import os

import torch
import torch.distributed as dist

from wav2vec2forbrain_amd import build_lib

if __name__ == "__main__":
    build_lib.ensure_built()     # a fresh checkout carries sources only
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("B2P_DIST_BACKEND", "nccl"))
    from wav2vec2forbrain_amd.args.argparsing import get_experiment_from_args
    experiment = get_experiment_from_args()
    experiment.run()
    if dist.is_initialized():
        dist.destroy_process_group()
