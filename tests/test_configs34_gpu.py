"""Adam trajectories against the ones the reference's own modules and optimizer produced
(tests/golden/make_golden.py: adam_trajectory): the bench workloads (base_bs32 = configs[1],
conformer_large_bs32 = configs[2]: 3 steps over the brain encoder, lr 1e-3, as bench.py's parity) and
BASELINE configs[3] and configs[4] on one GPU (their per-GPU workloads):

  large960_bs32           wav2vec2-large-960h (post-LN 1024/24L/16H/4096), GRU H256x2, fc [] (the
                          512 -> 1024 projection), 32 x 1024 bins; unfreeze_strategy=brain_encoder,
                          2 Adam steps (torch.optim.Adam, lr 1e-3).
  conformer_large_ft_bs8  Conformer-large, unfreeze_strategy=brain_encoder+w2v (two param groups,
                          b2t_gru_w2v_conformer_experiment.py:87-123: brain lr 1e-3, w2v lr 1e-4, L2
                          weight decay 1e-5), 8 x 1024 bins (two padded samples), 3 Adam steps over
                          all 618 M parameters.

The build runs them through Trainer.train_step (train/train_loop.py: the step run.py executes): the
first step eager, then the step is captured once and replayed, so the later steps are graph replays
— including the recast of the trained 16-bit weight copies inside the replay. Deterministic mode
(dropout / LayerDrop 0), in both precision modes:
  fp32  exact-fp32 MFMA: every step's loss tracks the reference's trajectory (FP32_TRAJ_RTOL).
  bf16  the default mode with the Trainer's precision policy: bf16 / fp16 operands, and the bf16x3 mode
        (split-bf16 GEMMs) when the w2v encoder itself is trained (configs[4]): Adam's first updates of
        its ~600 M parameters are ~lr * sign(g), and 16-bit operand rounding moved that trajectory's third
        loss 1.3e-3 .. 7.4e-3 off the reference's. Every step of every fixture is
        held to the north-star 1e-3; the sampled updates are compared by direction."""
import numpy as np
import pytest
import torch

from tests.helpers import CFG, load_fixture, build_model, batch_dict

pytestmark = pytest.mark.gpu

LOSS_RTOL = 1e-3        # BASELINE.json north_star: the loss at the reference's weights
FP32_TRAJ_RTOL = 1e-4   # exact-fp32 mode, every step of the trajectory
# Sign-weighted lost share of the reference's parameter updates per family (brain_encoder / w2v) after the
# first Adam update, printed by the test. Adam's first updates are ~lr * sign(g), so this is the share of
# the update magnitude whose direction the 16-bit rounding flipped. Measured (round 5): fp32 mode <= 1.2e-6;
# default mode brain_encoder 1.0e-3 / 1.8e-3 / 2.8e-3 (configs 1-3, bf16), configs[4] (bf16x3 policy) w2v
# 2.7e-6, brain_encoder 4.1e-7. The bf16 gate sits at ~1.8x the worst measured value (not at the north
# star's 1e-3, which bounds the loss, not this share).
SIGN_LOST_MAX = {"fp32": 1e-4, "bf16": 5e-3}
BF16_TRAJ_RTOL = {"base_bs32": 1e-3, "conformer_large_bs32": 1e-3, "large960_bs32": 1e-3,
                  "conformer_large_ft_bs8": 1e-3}
# the precision the policy picks per fixture (the w2v encoder trained -> bf16x3)
POLICY = {"base_bs32": None, "conformer_large_bs32": None, "large960_bs32": None, "conformer_large_ft_bs8": "bf16x3"}


def _trajectory(name, mode):
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    cfg = CFG[name]
    a = cfg["adam"]
    model = build_model(cfg)
    model.train()
    p0 = {n: p.detach().clone() for n, p in model.named_parameters()}
    exp = SyntheticStepExperiment(model, unfreeze="brain_encoder+w2v" if a["w2v_lr"] is not None else "brain_encoder",
                                  lr=a["lr"], w2v_lr=a["w2v_lr"], weight_decay=a["wd"])
    b = batch_dict(cfg)
    batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
    with Fn.precision(mode):
        trainer = Trainer(exp)
        trainer.capture_after = 1
        losses = [float(trainer.train_step(batch).loss) for _ in range(a["steps"])]
        assert trainer.step_precision() == (POLICY[name] if mode == "bf16" else None)
    torch.cuda.synchronize()
    assert trainer.eager_steps == 1 and trainer.graph_steps == a["steps"] - 1
    trainer.release_graphs()
    Fn.set_deferred_wgrad([])
    deltas = {n: (p.detach() - p0[n]).reshape(-1) for n, p in model.named_parameters()}
    return losses, deltas, trainer


@pytest.mark.parametrize("name", ["base_bs32", "conformer_large_bs32", "large960_bs32", "conformer_large_ft_bs8"])
@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_adam_trajectory_matches_reference(name, mode):
    fx = load_fixture(name)
    ref = [float(v) for v in fx["adam_losses"]]
    losses, deltas, trainer = _trajectory(name, mode)
    rel = [abs(g - r) / abs(r) for g, r in zip(losses, ref)]
    print(f"{name} [{mode}]: build {losses} reference {ref} rel {rel}")
    if mode == "fp32":
        assert max(rel) <= FP32_TRAJ_RTOL, (losses, ref, rel)
    else:
        assert rel[0] <= LOSS_RTOL, (losses, ref, rel)
        assert max(rel[1:]) <= BF16_TRAJ_RTOL[name], (losses, ref, rel)
    # parameter updates: every parameter the reference's Adam moved moved here by about as much, and
    # every parameter it left alone (unused inpLayer* / hidden_start / conformer pos_conv_embed:
    # grad None) stayed bit-identical
    worst = 0.0
    lost = {"brain_encoder": [0.0, 0.0], "w2v": [0.0, 0.0]}   # sign-weighted lost descent of the updates
    for n in fx["param_names"]:
        dref = float(fx["dnorm/" + n])
        d = deltas[n]
        if dref == 0.0:
            assert float(d.abs().max()) == 0.0, n
            continue
        if n.endswith(("attention.k_proj.bias", "self_attn.linear_k.bias")):
            continue   # its gradient is analytically zero (softmax is shift-invariant): pure rounding noise
        got = float(d.double().norm())
        worst = max(worst, abs(got - dref) / dref)
        v = d[torch.from_numpy(fx["didx/" + n]).cuda()].cpu().numpy()
        r = fx["dval/" + n]
        # Adam's first updates are ~lr * sign(g): entries whose gradient is near zero may flip sign
        # under bf16 rounding, so the sampled entries are compared by their correlation
        c = float(np.dot(v, r) / (np.linalg.norm(v) * np.linalg.norm(r) + 1e-30))
        assert c >= (0.99 if mode == "fp32" else 0.9), (n, c)
        # Adam's updates are ~lr * sign(m / sqrt(v)): the share of the reference's update magnitude whose
        # direction flipped here (the w2v updates of the full fine-tune, configs[4])
        part = lost["brain_encoder" if n.startswith("brain_encoder.") else "w2v"]
        part[0] += float(np.abs(r)[np.sign(v) != np.sign(r)].sum())
        part[1] += float(np.abs(r).sum())
    shares = {k: (a / b if b > 0 else 0.0) for k, (a, b) in lost.items()}
    print(f"{name} [{mode}]: worst relative update-norm error {worst:.3e}; sign-lost update share "
          + ", ".join(f"{k} {v:.2e}" for k, v in shares.items()))
    for k, v in shares.items():
        assert v <= SIGN_LOST_MAX[mode], (k, v)
    assert worst <= 0.1, worst
    # the optimizer's per-parameter step counters: one per update for every used parameter
    opt = trainer.optimizer
    opt.sync_steps()
    steps = {float(opt.state[p]["step"]) for g in opt.param_groups for p in g["params"]
             if len(opt.state[p]) and float(fx["dnorm/" + _name(trainer.model, p)]) > 0}
    assert steps == {float(CFG[name]["adam"]["steps"])}, steps


def _name(model, p):
    for n, q in model.named_parameters():
        if q is p:
            return n
    raise KeyError
