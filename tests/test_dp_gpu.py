"""Data-parallel identity on the real model: two ranks (gloo, both on
the one GPU of the box), each stepping half of a global batch through the HIP training step with
train.ddp.GradBucketReducer, produce the single-process global-batch loss (mean of the rank means)
and gradients (bucket average). For the Conformer this holds because BatchNorm statistics are
synchronised over the ranks (functional.sync_batchnorm); its running statistics match too.
Deterministic mode (dropout / LayerDrop 0), exact-fp32 MFMA, so only the reduction order differs."""
import math
import os
import socket

import pytest
import torch

from tests.helpers import CFG, build_model, batch_dict

pytestmark = pytest.mark.gpu

WORLD = 2


def _cfg(name):
    c = dict(CFG[name])
    c.update(name=name, B=4, in_lens=[c["L"], c["L"] - 16, c["L"] - 24, c["L"]])
    return c


def _batch(cfg, rows):
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    b = batch_dict(cfg)
    sl = slice(rows[0], rows[1])
    tl = b["target_lens"][sl]
    S = int(b["target_lens"].max())
    return make_b2t_batch(b["x"][sl], b["target"][sl, :S], b["day_idxs"][sl], b["input_lens"][sl], tl).cuda()


def _step(model, batch, reducer=None):
    from wav2vec2forbrain_amd import functional as Fn
    if reducer is not None:
        reducer.zero_grad()
    with Fn.precision("fp32"):
        out = model(batch)
        out.loss.backward()
        Fn.join_wgrad()
    if reducer is not None:
        reducer.finish()
    torch.cuda.synchronize()
    return float(out.metrics["ctc_loss"])


def _trainable(model):
    from wav2vec2forbrain_amd.train.ddp import unused_param_names
    skip = unused_param_names(model)
    return [(n, p) for n, p in model.named_parameters() if n.startswith("brain_encoder.") and n not in skip]


def _worker(rank, name, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from wav2vec2forbrain_amd.train.ddp import GradBucketReducer
        cfg = _cfg(name)
        model = build_model(cfg)
        model.train()
        for p in model.w2v_encoder.parameters():   # unfreeze=brain_encoder: w2v weights frozen
            p.requires_grad_(False)
        red = GradBucketReducer([p for _, p in _trainable(model)], bucket_mb=0.05)
        per = cfg["B"] // WORLD
        loss = _step(model, _batch(cfg, (rank * per, (rank + 1) * per)), red)
        loss_t = torch.tensor([loss])
        dist.all_reduce(loss_t)
        torch.save({"loss": float(loss_t) / WORLD,
                    "grads": {n: p.grad.detach().cpu() for n, p in _trainable(model)},
                    "bufs": {n: b.detach().cpu() for n, b in model.named_buffers() if b.is_floating_point()}},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name", ["tiny_a", "tiny_conf"])
def test_dp_step_equals_global_batch_step(name, tmp_path):
    import torch.multiprocessing as mp
    cfg = _cfg(name)
    ref = build_model(cfg)
    ref.train()
    for p in ref.w2v_encoder.parameters():
        p.requires_grad_(False)
    loss = _step(ref, _batch(cfg, (0, cfg["B"])))
    grads = {n: p.grad.detach().cpu() for n, p in _trainable(ref)}
    bufs = {n: b.detach().cpu() for n, b in ref.named_buffers() if b.is_floating_point()}

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, name, port, str(tmp_path))) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(WORLD)]
    for r in res:
        assert abs(r["loss"] - loss) <= 2e-5 * abs(loss), (r["loss"], loss)
        gmax = max(float(g.norm()) for g in grads.values())
        for n, g in grads.items():
            d = float((r["grads"][n] - g).norm())
            assert d <= 1e-4 * float(g.norm()) + 1e-6 * gmax, (n, d, float(g.norm()))
        for n, b in bufs.items():   # Conformer BatchNorm running stats: global-batch statistics (SyncBN)
            d = float((r["bufs"][n] - b).norm())
            assert d <= 1e-4 * float(b.norm()) + 1e-6, (n, d)
    # the ranks hold identical gradients after the exchange
    for n in grads:
        assert torch.equal(res[0]["grads"][n], res[1]["grads"][n]), n


def _trainer_steps(model, batches, graphs, unfreeze="brain_encoder"):
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    info = {}
    with Fn.precision("fp32"):
        trainer = Trainer(SyntheticStepExperiment(model, unfreeze=unfreeze, lr=1e-3))
        trainer.use_graphs = graphs
        trainer.capture_after = 1
        losses, logs = [], []
        for b in batches:
            if trainer.reducer is not None:
                trainer.reducer.launch_log.clear()
                trainer.reducer.launch_tail.clear()
                trainer.reducer.launch_pending.clear()
            losses.append(float(trainer.train_step(b).loss))
            if trainer.reducer is not None:   # per step: the bucket launches the host issued (capture included)
                logs.append((list(trainer.reducer.launch_log), list(trainer.reducer.launch_pending)))
    torch.cuda.synchronize()
    if trainer.reducer is not None:   # the last step's bucket launches (a replay when graphs are on)
        info.update(launch_log=list(trainer.reducer.launch_log), launch_tail=list(trainer.reducer.launch_tail),
                    buckets=len(trainer.reducer.buckets), step_logs=logs, nparams=len(trainer.reducer.params))
    info["segments"] = [g["graph"].segments for g in trainer._graphs.values()]
    counts = (trainer.eager_steps, trainer.graph_steps)
    trainer.release_graphs()
    Fn.set_deferred_wgrad([])
    return losses, counts, info


def _optimised(model, unfreeze):
    from wav2vec2forbrain_amd.train.ddp import unused_param_names
    if unfreeze == "brain_encoder":
        return _trainable(model)
    skip = unused_param_names(model)
    return [(n, p) for n, p in model.named_parameters() if n not in skip and p.requires_grad]


def _trainer_worker(rank, name, port, out_dir, unfreeze="brain_encoder", bucket_mb="64", eager_too=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), B2P_DP_BUCKET_MB=bucket_mb)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        cfg = _cfg(name)
        model = build_model(cfg)
        model.train()
        model.sync_metrics = False
        per = cfg["B"] // WORLD
        b = _batch(cfg, (rank * per, (rank + 1) * per))
        losses, counts, info = _trainer_steps(model, [b] * 3, graphs=True, unfreeze=unfreeze)
        rec = {"losses": losses, "counts": counts, "info": info,
               "params": {n: p.detach().cpu() for n, p in _optimised(model, unfreeze)},
               "bufs": {n: b.detach().cpu() for n, b in model.named_buffers() if b.is_floating_point()}}
        if eager_too:   # the same data-parallel steps without graphs, from the same initial model
            model = build_model(cfg)
            model.train()
            model.sync_metrics = False
            rec["eager_losses"] = _trainer_steps(model, [b] * 3, graphs=False, unfreeze=unfreeze)[0]
            rec["eager_params"] = {n: p.detach().cpu() for n, p in _optimised(model, unfreeze)}
        torch.save(rec, os.path.join(out_dir, f"trainer_rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_dp_replayed_trainer_steps_equal_global_batch_steps(tmp_path):
    """Data-parallel Trainer steps with replays (train/train_loop.py: step 1 eager, then forward +
    backward captured and replayed; after each replay the bucket all-reduce, the used-by-some-rank
    gates and the device-form Adam run): three steps of two ranks on half batches give the parameters
    of three single-process Trainer steps on the whole batch (fp32 MFMA, deterministic mode)."""
    import torch.multiprocessing as mp
    name = "tiny_a"
    cfg = _cfg(name)
    ref = build_model(cfg)
    ref.train()
    ref_losses, _, _ = _trainer_steps(ref, [_batch(cfg, (0, cfg["B"]))] * 3, graphs=False)
    params = {n: p.detach().cpu() for n, p in _trainable(ref)}

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, name, port, str(tmp_path))) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [torch.load(tmp_path / f"trainer_rank{r}.pt", weights_only=True) for r in range(WORLD)]
    for r in res:
        assert tuple(r["counts"]) == (1, 2), r["counts"]
    for k in range(3):   # the global-batch loss is the mean of the rank means
        glob = (res[0]["losses"][k] + res[1]["losses"][k]) / 2
        assert abs(glob - ref_losses[k]) <= 2e-5 * abs(ref_losses[k]), (k, glob, ref_losses[k])
    for n, p in params.items():
        for r in res:
            d = float((r["params"][n] - p).norm())
            assert d <= 1e-4 * float(p.norm()) + 1e-6, (n, d)
        assert torch.equal(res[0]["params"][n], res[1]["params"][n]), n


def test_dp_replayed_syncbn_full_ft_steps_equal_global_batch_steps(tmp_path):
    """The Conformer with synchronised BatchNorm, fully fine-tuned (unfreeze=brain_encoder+w2v), under
    data-parallel replays: the step is captured in segments split at every SyncBN statistics
    all-reduce (forward and backward) and at every gradient-bucket launch (train/step_graph.py), and a
    replay issues those collectives between the segments. Three steps of two ranks on half batches
    give the parameters and BatchNorm running statistics of three single-process steps on the whole
    batch, steps 2-3 are replays, and the replay launched gradient buckets with captured backward
    still to run after them (the exchange overlapped the backward)."""
    import torch.multiprocessing as mp
    name, unfreeze = "tiny_conf", "brain_encoder+w2v"
    cfg = _cfg(name)
    ref = build_model(cfg)
    ref.train()
    ref_losses, _, _ = _trainer_steps(ref, [_batch(cfg, (0, cfg["B"]))] * 3, graphs=False, unfreeze=unfreeze)
    params = {n: p.detach().cpu() for n, p in _optimised(ref, unfreeze)}
    bufs = {n: b.detach().cpu() for n, b in ref.named_buffers() if b.is_floating_point()}

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, name, port, str(tmp_path), unfreeze, "0.01", True))
             for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [torch.load(tmp_path / f"trainer_rank{r}.pt", weights_only=True) for r in range(WORLD)]
    for r in res:
        assert tuple(r["counts"]) == (1, 2), r["counts"]
        info = r["info"]
        nconv = sum(1 for n in bufs if n.endswith("running_mean"))
        # 3 SyncBN all-reduces per conv module (2 forward, 1 backward) + the bucket launch points
        assert info["segments"][0] >= 3 * nconv + 2, (info["segments"], nconv)
        assert info["buckets"] >= 3, info
        assert sorted(info["launch_log"]) == list(range(info["buckets"])), info
        assert max(info["launch_tail"]) > 0, info   # some bucket went out before the backward ended
    for k in range(3):
        glob = (res[0]["losses"][k] + res[1]["losses"][k]) / 2
        assert abs(glob - ref_losses[k]) <= 2e-5 * abs(ref_losses[k]), (k, glob, ref_losses[k])
    # the key-projection bias has no true gradient (softmax over keys ignores it): its gradient is
    # reduction noise that Adam normalises to +-lr, so it is compared replay-vs-eager only
    noise = [n for n in params if n.endswith("linear_k.bias")]
    glob, rep = {}, {}
    for n, p in params.items():
        for r in res:
            glob[n] = max(glob.get(n, 0.0), float((r["params"][n] - p).norm()) / float(p.norm()))
            rep[n] = max(rep.get(n, 0.0), float((r["params"][n] - r["eager_params"][n]).norm()) / float(p.norm()))
        assert torch.equal(res[0]["params"][n], res[1]["params"][n]), n
    print("rel param diff, replayed DP vs global batch:", sorted(glob.items(), key=lambda kv: -kv[1])[:6])
    print("rel param diff, replayed DP vs eager DP:", sorted(rep.items(), key=lambda kv: -kv[1])[:6])
    for n in params:
        assert rep[n] <= 1e-5, (n, rep[n])
        if n not in noise:
            assert glob[n] <= 2e-4, (n, glob[n])
    for n, b in bufs.items():
        for r in res:
            d = float((r["bufs"][n] - b).norm())
            assert d <= 1e-4 * float(b.norm()) + 1e-6, (n, d)


def _nccl_world1_worker(port, out_dir, graphs, in_graph):
    """One rank, backend nccl (RCCL), B2P_DP_FORCE=1: every data-parallel code path runs over RCCL."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), B2P_DP_FORCE="1",
                      B2P_GRAPH_COLLECTIVES="1" if in_graph else "0", B2P_DP_BUCKET_MB="0.05")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        cfg = _cfg("tiny_conf")
        model = build_model(cfg)
        model.train()
        model.sync_metrics = False
        b = _batch(cfg, (0, cfg["B"]))
        from wav2vec2forbrain_amd.train import ddp
        with_trainer = {}
        losses, counts, info = _trainer_steps(model, [b] * 3, graphs=graphs, unfreeze="brain_encoder+w2v")
        with_trainer.update(losses=losses, counts=counts, info=info, in_graph=ddp.collectives_in_graph(),
                            params={n: p.detach().cpu() for n, p in _optimised(model, "brain_encoder+w2v")})
        torch.save(with_trainer, os.path.join(out_dir, f"nccl_{int(graphs)}{int(in_graph)}.pt"))
    finally:
        dist.destroy_process_group()


def _single_process_ref_worker(out_dir):
    """The single-process reference steps of the RCCL world-1 test in a fresh process, like the workers
    (state earlier tests left in the pytest process, e.g. consumed dropout seeds, cannot reach it)."""
    torch.cuda.set_device(0)
    cfg = _cfg("tiny_conf")
    ref = build_model(cfg)
    ref.train()
    losses, _, _ = _trainer_steps(ref, [_batch(cfg, (0, cfg["B"]))] * 3, graphs=False, unfreeze="brain_encoder+w2v")
    torch.save({"losses": losses, "params": {n: p.detach().cpu() for n, p in _optimised(ref, "brain_encoder+w2v")}},
               os.path.join(out_dir, "single_process_ref.pt"))


def test_rccl_world1_captured_collectives(tmp_path):
    """BASELINE configs[3]/[4] run over RCCL on 8 GPUs, which this box cannot: a one-rank RCCL process
    group with the data-parallel machinery forced on (B2P_DP_FORCE=1) runs the Conformer's SyncBN
    statistics all-reduces, the gradient-bucket all-reduces and the used-flag MAX all-reduce through
    RCCL. Three full-fine-tune Trainer steps, eager, replayed with the collectives captured INSIDE one
    graph (the RCCL default, train.ddp.collectives_in_graph) and replayed with the segmented capture,
    leave the same parameters as the single-process steps (one rank: the all-reduces are identities)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_single_process_ref_worker, args=(str(tmp_path),))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0, p.exitcode
    ref = torch.load(tmp_path / "single_process_ref.pt", weights_only=True)
    ref_losses, params = ref["losses"], ref["params"]
    res = {}
    for graphs, in_graph in ((False, True), (True, True), (True, False)):
        p = ctx.Process(target=_nccl_world1_worker, args=(_free_port(), str(tmp_path), graphs, in_graph))
        p.start()
        p.join(timeout=240)
        assert p.exitcode == 0, (graphs, in_graph, p.exitcode)
        res[(graphs, in_graph)] = torch.load(tmp_path / f"nccl_{int(graphs)}{int(in_graph)}.pt", weights_only=True)
    for key, r in res.items():
        graphs, in_graph = key
        assert tuple(r["counts"]) == ((1, 2) if graphs else (3, 0)), (key, r["counts"])
        if graphs:
            # one graph per step with the collectives inside; one segment per collective otherwise
            assert (r["info"]["segments"][0] == 1) == in_graph, (key, r["info"]["segments"])
            assert r["in_graph"] == in_graph
        if graphs and in_graph:
            # the RCCL graph holds the whole exchange: the capture (step 2) launched every
            # bucket, the first while gradients of the backward were still to come (its all-reduce overlaps
            # the rest of the backward in every replay); a replay (step 3) issues nothing from the host
            cap_log, cap_pending = r["info"]["step_logs"][1]
            assert sorted(cap_log) == list(range(r["info"]["buckets"])), (key, cap_log)
            assert r["info"]["buckets"] > 1 and cap_pending[0] > 0, (key, cap_pending)
            assert r["info"]["step_logs"][2] == ([], []), (key, r["info"]["step_logs"][2])
        for k in range(3):
            assert abs(r["losses"][k] - ref_losses[k]) <= 1e-5 * abs(ref_losses[k]), (key, k, r["losses"], ref_losses)
        worst = max(float((r["params"][n] - q).norm()) / (float(q.norm()) + 1e-30) for n, q in params.items()
                    if not n.endswith("linear_k.bias"))
        print(key, "worst relative parameter difference vs single-process steps", worst)
        assert worst <= 1e-5, (key, worst)


def _ld_worker(rank, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from wav2vec2forbrain_amd import functional as Fn
        from wav2vec2forbrain_amd.train.train_loop import Trainer
        from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
        torch.manual_seed(1234)                        # the host LayerDrop draws of eager steps: equal on every rank
        Fn.SEEDS.reseed(99 + rank)                     # dropout masks differ per rank
        Fn.LD_SEEDS.reseed(4242)                       # device LayerDrop draws of replays: equal on every rank
        cfg = _cfg("tiny_a")
        model = build_model(cfg)
        model.train()
        model.sync_metrics = False
        enc = model.w2v_encoder.wav2vec2.encoder
        enc.config.layerdrop = 0.5
        ran = []
        for i, layer in enumerate(enc.layers):
            layer.register_forward_hook(lambda m, a, o, i=i: ran.append(i))
        per = cfg["B"] // WORLD
        b = _batch(cfg, (rank * per, (rank + 1) * per))
        record = []
        with Fn.precision("fp32"):
            trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
            trainer.capture_after = 2
            for _ in range(6):
                ran.clear()
                g0 = trainer.graph_steps
                trainer.train_step(b)
                torch.cuda.synchronize()
                if trainer.graph_steps > g0:   # a replay: this replay's device draw per layer
                    record.append(("replay", [int(f.item()) for f in Fn._GATE_FLAGS[-len(enc.layers):]]))
                else:
                    record.append(("eager", sorted(ran)))
        counts = (trainer.eager_steps, trainer.graph_steps)
        trainer.release_graphs()
        Fn.set_deferred_wgrad([])
        torch.save({"record": record, "counts": counts,
                    "params": {n: p.detach().cpu() for n, p in _trainable(model)}},
                   os.path.join(out_dir, f"ld_rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_dp_layerdrop_same_layers_on_every_rank(tmp_path):
    """Data-parallel steps at LayerDrop 0.5 (two gloo ranks on the one GPU): the eager steps (the host
    draw of the reference, torch.rand per layer from the rank-equal torch seed) and the replays (the
    device draw from LD_SEEDS, rank-equal, functional.layerdrop_layer) skip the same layers on both
    ranks, while the dropout masks differ per rank; the parameters stay identical across ranks."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_ld_worker, args=(r, port, str(tmp_path))) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [torch.load(tmp_path / f"ld_rank{r}.pt", weights_only=True) for r in range(WORLD)]
    assert tuple(res[0]["counts"]) == (2, 4), res[0]["counts"]
    assert res[0]["record"] == res[1]["record"], (res[0]["record"], res[1]["record"])
    kinds = [k for k, _ in res[0]["record"]]
    assert kinds == ["eager"] * 2 + ["replay"] * 4, kinds
    nl = _cfg("tiny_a")["layers"]
    skipped = sum(nl - len(v) for k, v in res[0]["record"] if k == "eager") + \
        sum(v.count(0) for k, v in res[0]["record"] if k == "replay")
    assert skipped > 0, res[0]["record"]   # the draws did skip layers (the test is not vacuous)
    for n in res[0]["params"]:
        assert torch.equal(res[0]["params"][n], res[1]["params"][n]), n


def _regroup_steps(model, batches, split):
    """Trainer steps whose optimizer starts with the first `split` brain-encoder parameters and gains
    the rest (HipAdam.add_param_group) after two steps; returns the losses."""
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.optim import HipAdam
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    ps = list(model.brain_encoder.parameters())

    class Exp(SyntheticStepExperiment):
        def create_optimizer(self):
            return HipAdam([{"params": ps[:split]}], lr=self.base_config.learning_rate)

    with Fn.precision("fp32"):
        trainer = Trainer(Exp(model, lr=1e-3))
        trainer.capture_after = 1
        losses = []
        for i, b in enumerate(batches):
            if i == 2:
                trainer.optimizer.add_param_group({"params": ps[split:]})
            losses.append(float(trainer.train_step(b).loss))
    torch.cuda.synchronize()
    counts = (trainer.eager_steps, trainer.graph_steps)
    trainer.release_graphs()
    Fn.set_deferred_wgrad([])
    return losses, counts


def _regroup_worker(rank, name, port, out_dir, split):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        cfg = _cfg(name)
        model = build_model(cfg)
        model.train()
        model.sync_metrics = False
        per = cfg["B"] // WORLD
        b = _batch(cfg, (rank * per, (rank + 1) * per))
        losses, counts = _regroup_steps(model, [b] * 4, split)
        torch.save({"losses": losses, "counts": counts,
                    "params": {n: p.detach().cpu() for n, p in _trainable(model)}},
                   os.path.join(out_dir, f"regroup_rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_dp_trainer_param_group_added_between_steps(tmp_path):
    """a param group added mid-run (HipAdam.add_param_group) under data parallelism.
    The Trainer rebuilds its bucket reducer, frozen reducer and optimizer gates for the new parameter set
    (train_loop.Trainer._setup_dp), so the new group's gradients are all-reduced: two ranks on half
    batches end with the parameters of the single-process global-batch run, and equal on both ranks."""
    import torch.multiprocessing as mp
    name = "tiny_a"
    cfg = _cfg(name)
    ref = build_model(cfg)
    ref.train()
    split = len(list(ref.brain_encoder.parameters())) // 2
    ref_losses, ref_counts = _regroup_steps(ref, [_batch(cfg, (0, cfg["B"]))] * 4, split)
    params = {n: p.detach().cpu() for n, p in _trainable(ref)}
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_regroup_worker, args=(r, name, port, str(tmp_path), split)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [torch.load(tmp_path / f"regroup_rank{r}.pt", weights_only=True) for r in range(WORLD)]
    for r in res:
        assert tuple(r["counts"]) == tuple(ref_counts) and r["counts"][1] >= 1, (r["counts"], ref_counts)
    for k in range(4):
        glob = (res[0]["losses"][k] + res[1]["losses"][k]) / 2
        assert abs(glob - ref_losses[k]) <= 2e-5 * abs(ref_losses[k]), (k, glob, ref_losses[k])
    for n, p in params.items():
        for r in res:
            d = float((r["params"][n] - p).norm())
            assert d <= 1e-4 * float(p.norm()) + 1e-6, (n, d)
        assert torch.equal(res[0]["params"][n], res[1]["params"][n]), n


def _capture_fallback_worker(port, out_dir):
    """One gloo rank with the data-parallel machinery forced on; every step capture raises."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), B2P_DP_FORCE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from wav2vec2forbrain_amd import functional as Fn
        from wav2vec2forbrain_amd.train.train_loop import Trainer
        from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
        cfg = _cfg("tiny_a")
        model = build_model(cfg)
        model.train()
        model.sync_metrics = False
        b = _batch(cfg, (0, cfg["B"]))
        with Fn.precision("fp32"):
            trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
            trainer.capture_after = 1

            def fail(batch):
                raise RuntimeError("capture refused (test)")
            trainer._capture = fail
            losses = [float(trainer.train_step(b).loss) for _ in range(3)]
        torch.save({"losses": losses, "counts": (trainer.eager_steps, trainer.graph_steps),
                    "failed": list(trainer._capture_failed.values())}, os.path.join(out_dir, "fallback.pt"))
        Fn.set_deferred_wgrad([])
    finally:
        dist.destroy_process_group()


def test_dp_capture_failure_falls_back_to_eager_steps(tmp_path):
    """A data-parallel step capture that raises leaves that batch shape on eager steps (the same update)
    instead of ending the run: every step eager, the capture tried once, finite losses."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_capture_fallback_worker, args=(_free_port(), str(tmp_path)))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0, p.exitcode
    r = torch.load(tmp_path / "fallback.pt", weights_only=True)
    assert tuple(r["counts"]) == (3, 0), r["counts"]
    assert len(r["failed"]) == 1 and "capture refused" in r["failed"][0], r["failed"]
    assert all(math.isfinite(v) for v in r["losses"]), r["losses"]
