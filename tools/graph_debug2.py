"""Debug: run-to-run determinism of the eager step, and host- vs device-hyper Adam after one step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from graph_debug import make, pdiff  # noqa: E402
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402

with Fn.precision("bf16"):
    runs = []
    for mode in ("host", "host", "dev"):
        m, o, s = make()
        if mode == "dev":
            o.make_capturable(torch.device("cuda"))
        l = float(s())
        torch.cuda.synchronize()
        runs.append((mode, m, l, {n: p.grad.clone() for n, p in m.brain_encoder.named_parameters() if p.grad is not None}))
    for i in (1, 2):
        ga, gb = runs[0][3], runs[i][3]
        worst = max((float((ga[n] - gb[n]).abs().max()), n) for n in ga)
        print(runs[0][0], "vs", runs[i][0], "loss", runs[0][2], runs[i][2], "grad max abs diff", worst,
              "param diff after 1 step", pdiff(runs[0][1], runs[i][1]))
