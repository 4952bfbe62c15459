"""hipBLASLt launches per eager and per replayed Trainer step of a bench config (which plain GEMMs the
library path takes inside the step). usage: python tools/blaslt_count.py [base|conformer]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from wav2vec2forbrain_amd import functional as Fn, _lib  # noqa: E402
from wav2vec2forbrain_amd.train.train_loop import Trainer  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "base"
cfg = bench.make_config(32, 1024, kind)
model = bench.build(cfg, "cuda")
model.train()
for m in model.modules():
    if hasattr(m, "sync_metrics"):
        m.sync_metrics = False
tr = Trainer(bench.experiment_for(kind, model))
tr.capture_after = 2
batch = bench.batch_on(cfg, "cuda")
lib = _lib.load()
Fn.GEMM_LOG = []
for i in range(5):
    lib.b2p_blaslt_calls(1)
    tr.train_step(batch)
    torch.cuda.synchronize()
    print(f"step {i} ({'replay' if tr.graph_steps and i >= 3 else 'eager/capture'}): {lib.b2p_blaslt_calls(1)} hipBLASLt launches",
          flush=True)
    if i == 0:
        log, Fn.GEMM_LOG = Fn.GEMM_LOG, None
        seen = {}
        for g in log:
            k = (g["M"], g["N"], g["K"], g["a16"], g["ak"], g["bk"], g["epi"], g["ksplit"], g["nz"])
            seen[k] = seen.get(k, 0) + 1
        for k, n in sorted(seen.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1]):
            print(f"  {n:3d} x M{k[0]} N{k[1]} K{k[2]} a16={k[3]} ak={k[4]} bk={k[5]} epi={k[6]} ks={k[7]} nz={k[8]}")
