"""Trainer.train_step with replayed steps (train/train_loop.py): per batch shape, the first step runs
eagerly, then the whole step (forward, CTC, backward, side-stream frozen-weight gradients, clip,
Adam) is captured once and replayed for every later batch of that shape, with the batch copied into
the captured step's static inputs. Checked against the same Trainer with replays switched off, on a
sequence that alternates two batch shapes (the capture cache) and changes the data between steps."""
import numpy as np
import pytest
import torch

from tests.helpers import CFG, build_model, batch_dict

pytestmark = pytest.mark.gpu


def _batches():
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    cfg = CFG["plumbing_base"]
    b = batch_dict(cfg)
    full = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
    # a second shape: 448 bins (the collate pads to the longest sample of a batch)
    crop = make_b2t_batch(b["x"][:, :448].contiguous(), b["target"], b["day_idxs"],
                          torch.tensor([448, 384]), b["target_lens"]).cuda()
    # same shape as `full`, other data: the replay must read the new batch
    flip = make_b2t_batch(b["x"].flip(0).contiguous(), b["target"].flip(0).contiguous(), b["day_idxs"].flip(0),
                          b["input_lens"].flip(0), b["target_lens"].flip(0)).cuda()
    return [full, full, crop, flip, crop, crop, full, flip]


@pytest.mark.parametrize("clip", [None, 0.5])
def test_trainer_replay_matches_eager(clip):
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    res = []
    for graphs in (False, True):
        model = build_model(CFG["plumbing_base"])
        model.train()
        with Fn.precision("bf16"):
            trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3, gradient_clipping=clip))
            trainer.use_graphs = graphs
            trainer.capture_after = 1
            losses, logits = [], []
            for batch in _batches():
                out = trainer.train_step(batch)
                losses.append(float(out.metrics["ctc_loss"]))
                logits.append(out.logits.detach().clone())
        torch.cuda.synchronize()
        if graphs:   # full: eager, replay x3 (flip shares its shape); crop: eager, replay x2
            assert (trainer.eager_steps, trainer.graph_steps, len(trainer._graphs)) == (2, 6, 2)
        trainer.optimizer.sync_steps()
        res.append((losses, logits, {n: p.detach().clone() for n, p in model.named_parameters()},
                    {n: p.grad.detach().clone() for n, p in model.named_parameters()
                     if not n.startswith("brain_encoder.") and p.grad is not None}))
        trainer.release_graphs()
        Fn.set_deferred_wgrad([])
    (la, ga, pa, fa), (lb, gb, pb, fb) = res
    np.testing.assert_allclose(lb, la, rtol=1e-5, atol=0)
    for x, y in zip(ga, gb):
        assert float((x - y).norm()) <= 1e-5 * float(x.norm())
    for n in pa:
        assert float((pa[n] - pb[n]).norm()) <= 1e-5 * float(pa[n].norm()) + 1e-7, n
    assert set(fa) == set(fb) and fa
    for n in fa:   # frozen w2v gradients keep accumulating across replays exactly as across eager steps
        assert float((fa[n] - fb[n]).norm()) <= 1e-5 * float(fa[n].norm()) + 1e-7, n
