"""bf16-mode CTC loss of a fixture vs the reference's, with the brain encoder's forward on fp16
operands (the default) and on bf16 operands (model.brain_forward_f16 / forward_f16 = False).
usage: python tools/brain16_probe.py <fixture> [...]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import CFG, build_model, load_fixture, batch_dict
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch

for name in sys.argv[1:]:
    cfg = CFG[name]
    ref = float(load_fixture(name)["loss"])
    b = batch_dict(cfg)
    batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
    for f16 in (True, False):
        model = build_model(cfg)
        model.train()
        if hasattr(model, "brain_forward_f16"):
            model.brain_forward_f16 = f16
        with torch.no_grad(), Fn.precision("bf16"):
            got = model(batch).metrics["ctc_loss"]
        print(f"{name} brain fp16={f16}: hip {got:.6f} ref {ref:.6f} rel {(got - ref) / abs(ref):+.3e}", flush=True)
        for n, m in model.named_modules():
            pass
        del model
