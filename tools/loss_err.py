"""bf16 HIP loss vs the fp32 CPU oracle at the BASELINE config (bs=32, L=1024, wav2vec2-base),
deterministic mode, with the persistent GRU on/off. usage: python tools/loss_err.py [B] [L]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import CFG, build_model, batch_dict, oracle_cfg
from oracle.b2p2t_oracle import forward_loss
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
L = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
cfg = dict(CFG["plumbing_base"], name="full_base", B=B, L=L, in_lens=[L] * B, tgt_range=(60, 120))
model = build_model(cfg)
model.train()
b = batch_dict(cfg)
batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
torch.set_num_threads(min(16, torch.get_num_threads()))
with torch.no_grad():
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ref = float(forward_loss(sd, b, oracle_cfg(cfg)))
for g16 in (0, 1):
    Fn._GRU16[0] = bool(g16)
    with torch.no_grad(), Fn.precision("bf16"):
        got = model(batch).metrics["ctc_loss"]
    print(f"B={B} L={L} GRU16={g16}: hip {got:.6f} oracle {ref:.6f} rel {abs(got - ref) / abs(ref):.2e}", flush=True)
