"""Bisects a crash in Trainer's step capture: each variant runs in its own subprocess (a segfault ends
only that variant). usage: python tools/trainer_capture_probe.py [variant ...]
variants: base, warm1, nodefer, noopt, nograd_none, fp32, syncdebug, direct, direct_static"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(variant):
    import torch
    from tests.helpers import CFG, build_model
    from tests.test_trainer_gpu import _batches
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train import step_graph
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    model = build_model(CFG["plumbing_base"])
    model.train()
    if variant == "warm1":
        orig = step_graph.StepGraph.__init__

        def init(self, fn, opt=None, warmup=2, warm_replays=2, epoch=None):
            orig(self, fn, opt, 1, warm_replays, epoch)
        step_graph.StepGraph.__init__ = init
    if variant == "syncdebug":
        import traceback
        import warnings
        orig_one = step_graph.StepGraph._one

        def one(self):
            torch.cuda.set_sync_debug_mode("error")
            try:
                return orig_one(self)
            except Exception:
                traceback.print_exc()
                raise
            finally:
                torch.cuda.set_sync_debug_mode(0)
        step_graph.StepGraph._one = one
    if variant.startswith("direct"):
        with Fn.precision("bf16"):
            trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
            batch = _batches()[0]
            trainer.train_step(batch)
            for m in model.modules():
                if hasattr(m, "sync_metrics"):
                    m.sync_metrics = False
            if variant == "direct_static":
                batch = batch.copy_and_change(**{f: getattr(batch, f).clone() for f in batch._fields
                                                 if isinstance(getattr(batch, f), torch.Tensor)})
                for a in ("day_idxs", "input_lens", "target_lens"):
                    v = getattr(_batches()[0], a, None)
                    if isinstance(v, torch.Tensor):
                        setattr(batch, a, v.clone())
            sg = step_graph.StepGraph(lambda: trainer._eager_body(batch, in_graph=True).loss.detach().reshape(1),
                                      trainer.optimizer, warmup=0, warm_replays=0)
            sg.capture()
            print(f"{variant}: captured, replay loss {float(sg.replay()):.5f}", flush=True)
            sg.release()
        print(f"{variant}: OK", flush=True)
        return
    with Fn.precision("fp32" if variant == "fp32" else "bf16"):
        trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
        trainer.capture_after = 1
        if variant == "nodefer":
            Fn.set_deferred_wgrad([])
        if variant == "noopt":
            real = trainer.optimizer.step
            trainer.optimizer.step = lambda *a, **k: (Fn.join_wgrad() if Fn.capturing() else real(*a, **k))
        if variant == "nograd_none":
            trainer.optimizer.zero_grad = lambda set_to_none=True: [p.grad.zero_() for g in trainer.optimizer.param_groups
                                                                     for p in g["params"] if p.grad is not None]
        for i, batch in enumerate(_batches()[:3]):
            out = trainer.train_step(batch)
            print(f"{variant}: step {i} loss {float(out.metrics['ctc_loss']):.5f} graphs {len(trainer._graphs)}",
                  flush=True)
    torch.cuda.synchronize()
    print(f"{variant}: OK", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        run(sys.argv[2])
        sys.exit(0)
    rc_all = 0
    for v in sys.argv[1:] or ["syncdebug", "direct", "direct_static"]:
        p = subprocess.run([sys.executable, "-u", __file__, "--one", v], timeout=240)
        print(f"== {v}: rc {p.returncode}", flush=True)
