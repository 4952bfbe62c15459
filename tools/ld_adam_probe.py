"""Step-by-step comparison of replayed LayerDrop steps with captured device-form Adam against eager
steps (host-form Adam) with the same skip pattern (tests/test_layerdrop_gpu.py): after every step,
the parameters / gradients that differ most. usage: python tools/ld_adam_probe.py [tiny_a|tiny_conf]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.test_layerdrop_gpu import _model, _batch, _ForcedRand, P_LD
from tests.helpers import CFG
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.optim import HipAdam
from wav2vec2forbrain_amd.train.step_graph import StepGraph

name = sys.argv[1] if len(sys.argv) > 1 else "tiny_a"
cfg = CFG[name]
Fn.SEEDS.reseed(4321)
model = _model(name)
ref = _model(name)
for m in ref.modules():
    if hasattr(m, "sync_metrics"):
        m.sync_metrics = True
batch = _batch(cfg)
opt = HipAdam(model.parameters(), lr=1e-2, weight_decay=1e-2)
ropt = HipAdam(ref.parameters(), lr=1e-2, weight_decay=1e-2)


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
    for k in range(4):
        lg = float(sg.replay())
        ep = int(sg.epoch.item())
        pat = tuple(Fn.layerdrop_keep(P_LD, s, ep) for s in seeds)
        ropt.zero_grad()
        forced = _ForcedRand(pat)
        torch.rand = forced
        try:
            out = ref(batch)
        finally:
            torch.rand = forced.orig
        out.loss.backward()
        gdiff = []
        rp = dict(ref.named_parameters())
        for n, p in model.named_parameters():
            e = rp[n].grad
            g = p.grad
            if e is None and g is None:
                continue
            e = torch.zeros_like(p) if e is None else e
            g = torch.zeros_like(p) if g is None else g
            gdiff.append((float((g - e).norm() / (e.norm() + 1e-30)), n))
        ropt.step()
        torch.cuda.synchronize()
        pdiff = sorted(((float((p - rp[n]).norm() / (rp[n].norm() + 1e-30)), n)
                        for n, p in model.named_parameters()), reverse=True)
        print(f"step {k}: pattern {pat} loss graph {lg:.6f} eager {float(out.metrics['ctc_loss']):.6f}")
        print("   worst grads:", [(f"{d:.2e}", n) for d, n in sorted(gdiff, reverse=True)[:4]])
        print("   worst params:", [(f"{d:.2e}", n) for d, n in pdiff[:4]], flush=True)
    sg.release()
