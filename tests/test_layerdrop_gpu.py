"""LayerDrop inside a captured training step (csrc/layerdrop.hip, functional.layerdrop_layer).

The reference redraws LayerDrop every step on the host (TF w2v Wav2Vec2Encoder.forward /
TF conf Wav2Vec2ConformerEncoder.forward: skip a layer when torch.rand([]) < layerdrop). A captured
step cannot redraw a host decision, so in a graph the draw is made on the device from the step
counter. These tests replay one captured step several times and check every replay against an eager
step that skips exactly the layers the device draw skipped in that replay: same loss, same
gradients, same Conformer BatchNorm running statistics (restored for skipped layers)."""
import numpy as np
import pytest
import torch

from tests.helpers import CFG, build_model, batch_dict

pytestmark = pytest.mark.gpu

P_LD = 0.5
REPLAYS = 8


def _batch(cfg):
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    b = batch_dict(cfg)
    return make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()


def _encoder(model):
    w = model.w2v_encoder
    return w.wav2vec2_conformer.encoder if hasattr(w, "wav2vec2_conformer") else w.wav2vec2.encoder


def _model(name):
    model = build_model(CFG[name])
    model.train()
    model.sync_metrics = False
    _encoder(model).config.layerdrop = P_LD
    return model


class _ForcedRand:
    """torch.rand([]) replacement for the eager reference: yields 0 (skip) / 0.99 (keep) per layer."""

    def __init__(self, pattern):
        self.vals = [0.99 if k else 0.0 for k in pattern]
        self.orig = torch.rand

    def __call__(self, *a, **kw):
        if len(a) == 1 and list(a[0]) == [] and not kw:
            return torch.tensor(self.vals.pop(0))
        return self.orig(*a, **kw)


@pytest.mark.parametrize("name", ["tiny_a", "tiny_conf"])
def test_captured_layerdrop_redraws_per_replay(name):
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.step_graph import StepGraph
    cfg = CFG[name]
    nl = cfg["layers"]
    Fn.SEEDS.reseed(1234)
    Fn.LD_SEEDS.reseed(1234)

    # ---- captured step, replayed
    model = _model(name)
    batch = _batch(cfg)

    def step():
        for p in model.parameters():
            p.grad = None
        out = model(batch)
        out.loss.backward()
        return out.metrics["ctc_loss"]

    Fn.LAYERDROP_LOG = []
    with Fn.precision("bf16"):
        sg = StepGraph(step, None, warmup=0, warm_replays=0)
        sg.capture()
        seeds = list(Fn.LAYERDROP_LOG)
        Fn.LAYERDROP_LOG = None
        assert len(seeds) == nl
        losses, patterns = [], []
        for _ in range(REPLAYS):
            losses.append(float(sg.replay()))
            ep = int(sg.epoch.item())
            patterns.append(tuple(Fn.layerdrop_keep(P_LD, s, ep) for s in seeds))
        grads_g = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        bufs_g = {n: b.detach().clone() for n, b in model.named_buffers() if b.is_floating_point()}
        counts_g = {n: int(b) for n, b in model.named_buffers() if n.endswith("num_batches_tracked")}
        sg.release()
    torch.cuda.synchronize()
    # the draw changes between replays (with p = 0.5 over REPLAYS replays)
    assert len(set(patterns)) > 1, patterns

    # ---- eager steps that skip the same layers
    ref = _model(name)
    for m in ref.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = True
    losses_e = []
    with Fn.precision("bf16"):
        for pat in patterns:
            for p in ref.parameters():
                p.grad = None
            forced = _ForcedRand(pat)
            torch.rand = forced
            try:
                out = ref(batch)
            finally:
                torch.rand = forced.orig
            out.loss.backward()
            losses_e.append(out.metrics["ctc_loss"])
    torch.cuda.synchronize()
    np.testing.assert_allclose(losses, losses_e, rtol=1e-5, atol=0)
    grads_e = {n: p.grad for n, p in ref.named_parameters() if p.grad is not None}
    for n, g in grads_g.items():
        e = grads_e.get(n)
        if e is None:   # a layer the last eager step skipped: the captured step wrote exact zeros
            assert float(g.abs().max()) == 0.0, n
            continue
        assert float((g - e).norm()) <= 1e-5 * float(e.norm()) + 1e-7, n
    for n, b in bufs_g.items():   # BatchNorm running statistics: updated only by kept layers
        e = dict(ref.named_buffers())[n]
        assert float((b - e).norm()) <= 1e-5 * float(e.norm()) + 1e-7, n
    # num_batches_tracked counts the replays that kept the layer (torch _BatchNorm.forward runs only then)
    counts_e = {n: int(b) for n, b in ref.named_buffers() if n.endswith("num_batches_tracked")}
    assert counts_g == counts_e and (not counts_g or len(set(counts_g.values())) > 1 or
                                     0 < min(counts_g.values()) < REPLAYS), (counts_g, counts_e)


@pytest.mark.parametrize("name", ["tiny_a", "tiny_conf"])
def test_captured_layerdrop_adam_leaves_dropped_layers(name):
    """Full fine-tuning under LayerDrop (config 5, unfreeze=brain_encoder+w2v): replayed steps with
    HipAdam over all parameters (device form: per-parameter step counters, the layer's LayerDrop gate
    on every tensor) vs eager steps with the same skip pattern, where a dropped layer's parameters
    have grad None and the update leaves them alone — value, both moments, L2 weight decay and the
    step count — as torch.optim.Adam does in the reference (src/experiments/experiment.py:25-28)."""
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.optim import HipAdam
    from wav2vec2forbrain_amd.train.step_graph import StepGraph
    cfg = CFG[name]
    Fn.SEEDS.reseed(4321)
    Fn.LD_SEEDS.reseed(4321)
    model = _model(name)
    batch = _batch(cfg)
    opt = HipAdam(model.parameters(), lr=1e-2, weight_decay=1e-2)

    def step():
        opt.zero_grad()
        out = model(batch)
        out.loss.backward()
        opt.step()
        return out.metrics["ctc_loss"]

    Fn.LAYERDROP_LOG = []
    with Fn.precision("bf16"):
        sg = StepGraph(step, opt, warmup=0, warm_replays=0)
        sg.capture()
        seeds = list(Fn.LAYERDROP_LOG)
        Fn.LAYERDROP_LOG = None
        losses, patterns = [], []
        for _ in range(REPLAYS):
            losses.append(float(sg.replay()))
            ep = int(sg.epoch.item())
            patterns.append(tuple(Fn.layerdrop_keep(P_LD, s, ep) for s in seeds))
        sg.release()
    torch.cuda.synchronize()
    opt.sync_steps()
    assert any(not all(p) for p in patterns), patterns     # some layer was dropped in some replay
    got = {n: (p.detach().clone(), opt.state[p]["exp_avg"].clone(), float(opt.state[p]["step"]))
           for n, p in model.named_parameters() if len(opt.state[p])}

    ref = _model(name)
    ropt = HipAdam(ref.parameters(), lr=1e-2, weight_decay=1e-2)
    losses_e = []
    with Fn.precision("bf16"):
        for pat in patterns:
            ropt.zero_grad()
            forced = _ForcedRand(pat)
            torch.rand = forced
            try:
                out = ref(batch)
            finally:
                torch.rand = forced.orig
            out.loss.backward()
            ropt.step()
            losses_e.append(float(out.metrics["ctc_loss"]))
    torch.cuda.synchronize()
    np.testing.assert_allclose(losses, losses_e, rtol=1e-5, atol=0)
    used_layers = [sum(p[k] for p in patterns) for k in range(cfg["layers"])]
    for n, p in ref.named_parameters():
        st = ropt.state[p]
        e_step = float(st["step"]) if len(st) else 0.0
        g_p, g_m, g_step = got[n] if n in got else (p.detach(), None, 0.0)
        assert g_step == e_step, (n, g_step, e_step)
        assert float((g_p - p.detach()).norm()) <= 1e-5 * float(p.detach().norm()) + 1e-7, n
        if len(st):
            assert float((g_m - st["exp_avg"]).norm()) <= 1e-5 * float(st["exp_avg"].norm()) + 1e-9, n
        if ".layers." in n:   # an encoder layer's tensors stepped once per replay that kept the layer
            k = int(n.split(".layers.")[1].split(".")[0])
            assert e_step == used_layers[k], (n, e_step, used_layers[k])


@pytest.mark.parametrize("name", ["tiny_a", "tiny_conf", "tiny_stable"])
def test_layerdrop_skip_gradient_fold_bitwise(name):
    """The skip-path gradient of a LayerDrop-selected layer is added inside the layer's input-gradient
    LayerNorm backward (functional._SkipSlot, b2p_layernorm_bwd_acc2) instead of by autograd in a
    separate add: replayed steps with and without the fold give bitwise-equal losses and gradients
    (exactly one of the two summands is nonzero in every replay), and the fold really removes the
    skip gradient from autograd (every layer's select hands it to a claiming Function)."""
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.step_graph import StepGraph
    cfg = CFG[name]
    out = {}
    for fold in (True, False):
        Fn._LD_SKIP_FOLD = fold
        Fn.SEEDS.reseed(99)
        Fn.LD_SEEDS.reseed(99)
        torch.manual_seed(3)
        model = _model(name)
        batch = _batch(cfg)
        slots = []
        orig = Fn._LayerDropSelect.apply

        def spy(x, y, p, seed, slot=None):
            slots.append(slot)
            return orig(x, y, p, seed, slot)

        def step():
            for p in model.parameters():
                p.grad = None
            o = model(batch)
            o.loss.backward()
            return o.metrics["ctc_loss"]

        Fn._LayerDropSelect.apply = spy
        try:
            with Fn.precision("bf16"):
                sg = StepGraph(step, None, warmup=0, warm_replays=0)
                sg.capture()
                losses = [float(sg.replay()) for _ in range(REPLAYS)]
                grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
                sg.release()
        finally:
            Fn._LayerDropSelect.apply = orig
            Fn._LD_SKIP_FOLD = True
        torch.cuda.synchronize()
        assert len(slots) == cfg["layers"]
        assert all((s is not None) == fold for s in slots), slots
        out[fold] = (losses, grads)
    assert out[True][0] == out[False][0]
    assert out[True][1].keys() == out[False][1].keys()
    for n, g in out[True][1].items():
        assert torch.equal(g, out[False][1][n]), n
