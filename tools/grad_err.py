"""Worst per-parameter gradient relative-L2 error (bf16 HIP step vs reference golden vectors).
usage: python tools/grad_err.py <fixture name> [mode]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.helpers import CFG, load_fixture, build_model, batch_dict
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch

name = sys.argv[1]
mode = sys.argv[2] if len(sys.argv) > 2 else "bf16"
cfg = CFG[name]
fx = load_fixture(name)
model = build_model(cfg)
model.train()
b = batch_dict(cfg)
batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
with Fn.precision(mode):
    out = model(batch)
    out.loss.backward()
torch.cuda.synchronize()
params = dict(model.named_parameters())
errs = []
for n in fx["param_names"]:
    g = params[n].grad if params[n].grad is not None else torch.zeros_like(params[n])
    if "grad/" + n in fx:
        r, v = fx["grad/" + n], g.cpu().numpy()
    else:
        r = fx["gval/" + n]
        v = g.reshape(-1)[torch.from_numpy(fx["gidx/" + n]).cuda()].cpu().numpy()
    errs.append((float(np.linalg.norm(v - r) / (np.linalg.norm(r) + 1e-30)), n))
errs.sort(reverse=True)
lg = out.logits.detach().cpu().numpy()
print(f"{name} {mode} GRU16={os.environ.get('B2P_GRU16', '1')}: loss rel "
      f"{abs(out.metrics['ctc_loss'] - float(fx['loss'])) / abs(float(fx['loss'])):.2e} logits relL2 "
      f"{np.linalg.norm(lg - fx['logits']) / np.linalg.norm(fx['logits']):.2e}; worst grads: "
      + ", ".join(f"{e:.3f} {n.split('.')[-3:]}" for e, n in errs[:4]), flush=True)
