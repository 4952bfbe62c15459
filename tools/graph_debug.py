"""Debug: eager vs device-hyper Adam vs graph replay on the plumbing_base config (dropout off)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.helpers import CFG, build_model  # noqa: E402
from tests.test_model_gpu import _batch  # noqa: E402
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402
from wav2vec2forbrain_amd.optim import HipAdam  # noqa: E402
from wav2vec2forbrain_amd.train.step_graph import StepGraph  # noqa: E402


def make(defer=True):
    cfg = CFG["plumbing_base"]
    model = build_model(cfg)
    model.train()
    for m in model.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = False
    opt = HipAdam(model.brain_encoder.parameters(), lr=1e-3)
    frozen = [p for n, p in model.named_parameters() if not n.startswith("brain_encoder.")]
    batch = _batch(cfg)

    def step():
        Fn.set_deferred_wgrad(frozen if defer else [])
        opt.zero_grad()
        out = model(batch)
        out.loss.backward()
        Fn.join_wgrad()
        opt.step()
        return out.metrics["ctc_loss"]
    return model, opt, step


def pdiff(a, b):
    worst = max(((float((pa - pb).norm()) / (float(pa.norm()) + 1e-12), n) for (n, pa), (_, pb) in
                 zip(a.named_parameters(), b.named_parameters())), default=(0, ""))
    return worst


if __name__ == "__main__":
  with Fn.precision("bf16"):
      A, oa, sa = make()
      la = [float(sa()) for _ in range(3)]
      B, ob, sb = make()
      ob.make_capturable(torch.device("cuda"))
      lb = [float(sb()) for _ in range(3)]
      torch.cuda.synchronize()
      print("eager host-Adam losses", la)
      print("eager dev-Adam  losses", lb, "param worst rel diff", pdiff(A, B))
      C, oc, sc = make()
      g = StepGraph(sc, oc, warmup=2)
      g.capture()
      print("after capture warmup: param diff vs A(after 3)", pdiff(A, C))
      l3 = float(g.replay())
      print("replay loss", l3, "vs eager step-3 loss", la[2])
      D, od, sd = make()
      sd(); sd()
      print("eager 2 steps vs C params after warmup+1 replay:", pdiff(D, C))
