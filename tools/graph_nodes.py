"""Autograd-graph census of one bench forward (GPU): the nodes whose output feeds several consumers (the
backward sums their incoming gradients with a torch add kernel) and the parameters accumulated by
autograd (AccumulateGrad: a torch add once .grad exists) rather than by the package's deferred
side-stream accumulation. usage: python tools/graph_nodes.py [base|conformer]"""
import collections
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.train.train_loop import Trainer
from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment, bench_config, build_model, device_batch

kind = sys.argv[1] if len(sys.argv) > 1 else "base"
cfg = bench_config(kind)
model = build_model(cfg, "cuda")
model.train()
for m in model.modules():
    if hasattr(m, "sync_metrics"):
        m.sync_metrics = False
Trainer(SyntheticStepExperiment(model, lr=1e-3))   # sets the deferred (frozen) parameter set
batch = device_batch(cfg, "cuda")
names = {id(p): n for n, p in model.named_parameters()}
with Fn.precision("bf16"):
    out = model(batch)
consumers = collections.Counter()
seen, stack = set(), [out.loss.grad_fn]
while stack:
    f = stack.pop()
    if f is None or f in seen:
        continue
    seen.add(f)
    for nf, _ in f.next_functions:
        if nf is not None:
            consumers[nf] += 1
            stack.append(nf)
print(f"[{kind}] {len(seen)} nodes")
for f, n in consumers.items():
    if n > 1:
        v = getattr(f, "variable", None)
        print(f"  {n} consumers: {type(f).__name__} {names.get(id(v), '') if v is not None else ''}")
acc = [f for f in seen if type(f).__name__ == "AccumulateGrad"]
dfr = [f for f in acc if Fn._defer_ok(f.variable)]
print(f"  AccumulateGrad nodes: {len(acc)} ({len(dfr)} of frozen parameters)")
