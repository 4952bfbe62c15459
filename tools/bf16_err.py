"""bf16-mode vs fp32-mode (exact-fp32 MFMA, matches the reference to 2e-5) CTC loss of the build on
the same weights and batch, deterministic mode. usage: python tools/bf16_err.py <base|conformer> [B] [L]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from wav2vec2forbrain_amd import functional as Fn

kind = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
L = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
cfg = bench.make_config(B, L, kind)
model = bench.build(cfg, "cuda", train_dropouts=False)
model.train()
batch = bench.batch_on(cfg, "cuda")
res = {}
for mode in ("fp32", "bf16"):
    with torch.no_grad(), Fn.precision(mode):
        res[mode] = model(batch).metrics["ctc_loss"]
rel = abs(res["bf16"] - res["fp32"]) / abs(res["fp32"])
print(f"{kind} B={B} L={L}: fp32 {res['fp32']:.6f} bf16 {res['bf16']:.6f} rel {rel:.2e}", flush=True)
