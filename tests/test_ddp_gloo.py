"""World-size-2 data-parallel gradient exchange on CPU (gloo): train/ddp.GradBucketReducer averages
every trainable gradient over the ranks, in both its modes — buckets all-reduced from the backward
hooks (eager step) and all buckets exchanged after backward (the graph-replayed step) — with
parameters that got no gradient on a rank contributing zeros, the collectives issued in the same
(index) order on every rank although one rank's backward never reaches a parameter, and gradients
accumulated either into bucket views (zero_grad) or into fresh tensors (copied in)."""
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
    extra = torch.nn.Linear(8, 8)      # a separate module, used on rank 0 only (registered last, so
    return m, extra                    # its parameters land in bucket 0, the first one launched)


def _params(mm):
    m, extra = mm
    return list(m.parameters()) + list(extra.parameters())


def _loss(mm, rank, x):
    m, extra = mm
    y = m(x)
    if rank == 0:
        y = extra(y)
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
        params = _params(m)
        red = GradBucketReducer(params, bucket_mb=0.001, overlap=overlap)   # several small buckets
        for it in range(3):                                                  # reusable across steps
            if it == 0:
                for p in params:          # fresh gradient tensors: copied into the buckets
                    p.grad = None
            else:
                red.zero_grad()           # gradients accumulate straight into the bucket views
            red.launch_log.clear()
            _loss(m, rank, _data(rank)).backward()
            red.finish()
            if it > 0:
                assert all(p.grad.data_ptr() == red.views[p].data_ptr() for p in params)
        order = list(red.launch_log)
        # expected: mean over ranks of each rank's own gradient (zeros where a rank had none)
        exp = []
        for r in range(world):
            mr = _model()
            _loss(mr, r, _data(r)).backward()
            exp.append([p.grad if p.grad is not None else torch.zeros_like(p) for p in _params(mr)])
        ok = all(torch.allclose(p.grad, sum(e[i] for e in exp) / world, rtol=1e-5, atol=1e-7)
                 for i, p in enumerate(params))
        q.put((rank, ok, len(red.buckets), order))
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
    assert all(ok for _, ok, _, _ in res), res
    assert all(nb > 1 for _, _, nb, _ in res)
    # identical collective order on both ranks: bucket index order
    assert all(order == list(range(nb)) for _, _, nb, order in res), res


def _gate_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wav2vec2forbrain_amd.train.ddp import GradBucketReducer
        torch.manual_seed(0)
        a, b, c = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)
        params = list(a.parameters()) + list(b.parameters()) + list(c.parameters())
        red = GradBucketReducer(params, bucket_mb=0.001)
        out = {}
        # eager step: the backward hooks mark what this rank used; a is used by both ranks, b by rank 0
        # only, c by neither (every rank's LayerDrop dropped its layer)
        red.zero_grad()
        x = torch.randn(2, 4)
        y = a(x)
        if rank == 0:
            y = b(y)
        y.sum().backward()
        red.finish()
        out["eager"] = [int(red.gates[id(p)]) for p in params]
        # replayed step: no hook fires; the used flags are the layers' device gates of this replay
        # (rank 0 kept layer b, rank 1 kept layer c; a has no gate: always used)
        fb = torch.tensor([1 if rank == 0 else 0], dtype=torch.int32)
        fc = torch.tensor([0 if rank == 0 else 1], dtype=torch.int32)
        st = red.make_layer_gates({**{id(p): fb for p in b.parameters()}, **{id(p): fc for p in c.parameters()}})
        red.use_layer_gates(st)
        red.zero_grad()
        red.finish()
        out["replay"] = [int(red.gates[id(p)]) for p in params]
        fc.fill_(0)   # next replay: nobody kept c
        red.zero_grad()
        red.finish()
        out["replay2"] = [int(red.gates[id(p)]) for p in params]
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_reducer_used_gates_world2_gloo():
    """The optimizer gates GradBucketReducer publishes (HipAdam's device form skips a gate-0 tensor,
    as torch.optim.Adam skips grad=None): "some rank used this parameter in this step", from the
    backward hooks in eager steps and from the device LayerDrop flags in replayed steps, MAX-reduced."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gate_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r]["eager"] == [1, 1, 1, 1, 0, 0], res
        assert res[r]["replay"] == [1, 1, 1, 1, 1, 1], res
        assert res[r]["replay2"] == [1, 1, 1, 1, 0, 0], res


def _regroup_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wav2vec2forbrain_amd.train.ddp import GradBucketReducer
        m = _model()
        params = _params(m)
        first = params[:2]   # the first param group; the rest joins later (add_param_group)
        red = GradBucketReducer(first, bucket_mb=0.001)
        red.zero_grad()
        _loss(m, rank, _data(rank)).backward()
        red.finish()
        # the Trainer's rebuild: the old reducer lets go of its parameters, a new one takes all of them
        red.close()
        for p in params:
            p.grad = None
        red2 = GradBucketReducer(params, bucket_mb=0.001)
        red2.zero_grad()
        red.launch_log.clear()
        _loss(m, rank, _data(rank)).backward()
        red2.finish()
        exp = []
        for r in range(world):
            mr = _model()
            _loss(mr, r, _data(r)).backward()
            exp.append([p.grad if p.grad is not None else torch.zeros_like(p) for p in _params(mr)])
        ok = all(torch.allclose(p.grad, sum(e[i] for e in exp) / world, rtol=1e-5, atol=1e-7)
                 for i, p in enumerate(params))
        q.put((rank, ok, len(red.launch_log), list(red2.launch_log) == list(range(len(red2.buckets)))))
    finally:
        dist.destroy_process_group()


def test_reducer_rebuilt_for_a_new_param_group_world2_gloo():
    """when the optimizer gains a param group under data parallelism the Trainer replaces its
    reducers (train_loop.Trainer._setup_dp). The replaced reducer's hooks are gone (it launches nothing
    more) and the new one averages every parameter, the new group's included."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_regroup_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, old_launches, in_order in res:
        assert ok and old_launches == 0 and in_order, res
