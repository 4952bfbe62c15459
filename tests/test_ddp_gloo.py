"""World-size-2 data-parallel gradient exchange on CPU (gloo): train/ddp.GradBucketReducer averages
every trainable gradient over the ranks, in both its modes — buckets all-reduced from the backward
hooks (eager step) and all buckets exchanged after backward (the graph-replayed step) — with
parameters that got no gradient on a rank contributing zeros."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 8))
    m.extra = torch.nn.Linear(8, 8)      # used on rank 0 only
    return m


def _loss(m, rank, x):
    y = m(x)
    if rank == 0:
        y = m.extra(y)
    return (y ** 2).mean()


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(5, 16, generator=g)


def _worker(rank, world, port, overlap, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wav2vec2forbrain_amd.train.ddp import GradBucketReducer
        m = _model()
        params = list(m.parameters())
        red = GradBucketReducer(params, bucket_mb=0.001, overlap=overlap)   # several small buckets
        for _ in range(2):                                                   # reusable across steps
            for p in params:
                p.grad = None
            _loss(m, rank, _data(rank)).backward()
            red.finish()
        # expected: mean over ranks of each rank's own gradient (zeros where a rank had none)
        exp = []
        for r in range(world):
            mr = _model()
            _loss(mr, r, _data(r)).backward()
            exp.append([p.grad if p.grad is not None else torch.zeros_like(p) for p in mr.parameters()])
        ok = all(torch.allclose(p.grad, sum(e[i] for e in exp) / world, rtol=1e-5, atol=1e-7)
                 for i, p in enumerate(params))
        q.put((rank, ok, len(red.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_grad_bucket_reducer_world2_gloo(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, overlap, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(nb > 1 for _, _, nb in res)
