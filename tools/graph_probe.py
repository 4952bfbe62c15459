"""Host launch time vs wall time of replayed Trainer steps, for a first and a second captured graph in one
process (the second graph's replays measured slower; is the host the bottleneck?).
usage: python tools/graph_probe.py [kind]   (kind: conformer (default) | base)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402
from wav2vec2forbrain_amd.train.train_loop import Trainer  # noqa: E402
from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "conformer"
Fn.set_precision("bf16")
for run in range(2):
    cfg = bench.make_config(32, 1024, kind)
    model = bench.build(cfg, "cuda")
    model.train()
    for m in model.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = False
    trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
    trainer.capture_after = 2
    batch = bench.batch_on(cfg, "cuda")
    for _ in range(3):
        trainer.train_step(batch)
    torch.cuda.synchronize()
    g = next(iter(trainer._graphs.values()))["graph"]
    host = []
    t0 = time.perf_counter()
    for _ in range(8):
        h0 = time.perf_counter()
        g.graph.replay()
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{kind} graph {run}: host replay launch {sum(host) / 8 * 1e3:.2f} ms each (first {host[0] * 1e3:.2f}), "
          f"issue loop {(t1 - t0) * 1e3:.1f} ms, wall {(t2 - t0) / 8 * 1e3:.2f} ms/step", flush=True)
    trainer.release_graphs()
    Fn.set_deferred_wgrad([])
    del trainer, model, batch, g
    bench.free_device()
