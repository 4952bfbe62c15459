"""bf16-mode CTC loss of a fixture vs the reference's, with blocks switched to exact fp32 (forward and
backward; Fn._FP32_OPS): which part of the model carries the loss error.
usage: python tools/fixture_err2.py <fixture> <ops,ops+ops,...>   (e.g. -,gru+linear+front)"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import CFG, build_model, load_fixture, batch_dict
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch

name = sys.argv[1]
cfg = CFG[name]
ref = float(load_fixture(name)["loss"])
b = batch_dict(cfg)
batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
model = build_model(cfg)
model.train()
for v in sys.argv[2].split(","):
    Fn._FP32_OPS.clear()
    Fn._FP32_OPS.update([] if v == "-" else v.split("+"))
    with torch.no_grad(), Fn.precision("bf16"):
        got = model(batch).metrics["ctc_loss"]
    print(f"{name} fp32[{v}]: hip {got:.6f} ref {ref:.6f} rel {(got - ref) / abs(ref):+.3e}", flush=True)
Fn._FP32_OPS.clear()
with torch.no_grad(), Fn.precision("fp32"):
    got = model(batch).metrics["ctc_loss"]
print(f"{name} all-fp32: hip {got:.6f} ref {ref:.6f} rel {(got - ref) / abs(ref):+.3e}", flush=True)
