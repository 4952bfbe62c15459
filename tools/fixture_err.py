"""bf16-mode CTC loss of the build vs a reference fixture's loss (tests/golden/<name>.npz), with each
block's forward switched to exact fp32 in turn (Fn._FP32_OPS) to attribute the error.
usage: python tools/fixture_err.py <fixture> [<fixture> ...]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import CFG, build_model, load_fixture
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
from tests.helpers import batch_dict

for name in sys.argv[1:]:
    cfg = CFG[name]
    fx = load_fixture(name)
    ref = float(fx["loss"])
    model = build_model(cfg)
    model.train()
    b = batch_dict(cfg)
    batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
    for ops in ("", "attn", "ffn", "conv", "linear", "gru", "attn,ffn,conv"):
        Fn._FP32_OPS.clear()
        Fn._FP32_OPS.update(filter(None, ops.split(",")))
        with torch.no_grad(), Fn.precision("bf16"):
            got = model(batch).metrics["ctc_loss"]
        print(f"{name} fp32[{ops or '-'}]: hip {got:.6f} ref {ref:.6f} rel {(got - ref) / abs(ref):+.3e}", flush=True)
    Fn._FP32_OPS.clear()
    with torch.no_grad(), Fn.precision("fp32"):
        got = model(batch).metrics["ctc_loss"]
    print(f"{name} all-fp32: hip {got:.6f} ref {ref:.6f} rel {(got - ref) / abs(ref):+.3e}", flush=True)
    del model
    torch.cuda.empty_cache()
