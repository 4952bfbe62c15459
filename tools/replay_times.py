"""Per-replay wall times of the captured bench step (synchronised after each), to see warm-up effects."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402
from wav2vec2forbrain_amd.optim import HipAdam  # noqa: E402
from wav2vec2forbrain_amd.train.step_graph import StepGraph  # noqa: E402

Fn.set_precision("bf16")
cfg = bench.make_config(32, 1024, "base")
model = bench.build(cfg, "cuda")
model.train()
for m in model.modules():
    if hasattr(m, "sync_metrics"):
        m.sync_metrics = False
opt = HipAdam(model.brain_encoder.parameters(), lr=1e-3)
Fn.set_deferred_wgrad([p for n, p in model.named_parameters() if not n.startswith("brain_encoder.")])
batch = bench.batch_on(cfg, "cuda")


def step():
    opt.zero_grad()
    out = model(batch)
    out.loss.backward()
    Fn.join_wgrad()
    opt.step()
    return out.metrics["ctc_loss"]


for _ in range(3):
    step()
torch.cuda.synchronize()
sg = StepGraph(step, opt)
sg.capture()
ts = []
for i in range(40):
    t0 = time.perf_counter()
    sg.replay()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print("per-replay ms:", " ".join(f"{t:.2f}" for t in ts))
t0 = time.perf_counter()
for i in range(40):
    sg.replay()
torch.cuda.synchronize()
print("40 back-to-back replays: %.3f ms/step" % ((time.perf_counter() - t0) * 1e3 / 40))
