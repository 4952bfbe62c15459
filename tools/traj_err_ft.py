"""Attribution of the bf16-mode trajectory error on a golden Adam-trajectory fixture with the w2v
encoder trained (VERDICT r4 "next" 1: configs[4] per GPU, conformer_large_ft_bs8).

For each variant, against the exact-fp32 mode of the same model on the same batch:
  * the step-1 gradient of every trained parameter, split into the brain encoder and the w2v encoder
    (and the w2v encoder by block kind): relative L2 error, the sign-descent efficiency
    (sum g_ref * sign(g) / sum |g_ref|: Adam's first update is ~lr * sign(g)) and the fraction of
    entries whose sign differs (each such entry is moved by a full lr the wrong way);
  * the CTC losses of the fixture's deterministic Adam steps (the fixture's param groups, lr, weight
    decay), relative to the reference's own trajectory stored in the fixture.
usage: python tools/traj_err_ft.py [fixture] [variant,variant,...]
variants: '-' plain bf16; 'B:attn+ffn' those blocks' backward in exact fp32 (forward unchanged);
'X:name' = a Fn.DIAG_SWITCHES switch; 'M:<mode>' = the whole step in precision mode <mode> (bf16x3); 'E:<bwd>:<S>' = forward in exact fp32, the Conformer blocks'
backward as <bwd> (b16: the 16-bit-operand backward; p16 / h16: the fp32-operand backward with every
GEMM operand rounded to bf16 / fp16; f32: exact fp32) on the loss scaled by S (gradients unscaled
before Adam): what fp16 backward operands with a static gradient scale would buy."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.helpers import CFG, load_fixture, build_model, batch_dict
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
from wav2vec2forbrain_amd.train.train_loop import Trainer
from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment

name = sys.argv[1] if len(sys.argv) > 1 else "conformer_large_ft_bs8"
variants = (sys.argv[2] if len(sys.argv) > 2 else "-,B:attn,B:ffn,B:conv,B:attn+ffn+conv").split(",")
cfg = CFG[name]
fx = load_fixture(name)
ref_losses = [float(v) for v in fx["adam_losses"]]
a = cfg["adam"]
b = batch_dict(cfg)
batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()


def kind_of(n):
    if n.startswith("brain_encoder."):
        return "brain"
    for k in ("self_attn.", "ffn1.", "ffn2.", "conv_module.", "attention.", "feed_forward."):
        if k in n:
            return k.rstrip(".")
    return "w2v_other"


def run(mode, bwd_only=(), switches=(), emul=None):
    Fn._FP32_OPS.clear()
    Fn._FP32_BWD_ONLY.clear()
    Fn._FP32_BWD_ONLY.update(bwd_only)
    for s in switches:
        Fn.DIAG_SWITCHES.add(s)
    model = build_model(cfg)
    model.train()
    exp = SyntheticStepExperiment(model, unfreeze="brain_encoder+w2v" if a["w2v_lr"] is not None else "brain_encoder",
                                  lr=a["lr"], w2v_lr=a["w2v_lr"], weight_decay=a["wd"])
    if emul is not None:
        bwd, S = emul
        trainer = Trainer(exp)
        if bwd != "b16":
            Fn.DIAG_SWITCHES.add("bwd32path")
        if bwd == "h16":
            Fn.DIAG_SWITCHES.add("bwdf16")

        def fb():
            trainer.optimizer.zero_grad()
            with Fn.precision("fp32"):
                out = model(batch)
            with Fn.precision("fp32" if bwd == "f32" else "bf16"):
                (out.loss * S).backward()
                Fn.join_wgrad()
            for p in model.parameters():
                if p.grad is not None:
                    p.grad.mul_(1.0 / S)
            return float(out.loss)
        fb()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        model.zero_grad(set_to_none=True)
        losses = []
        for _ in range(a["steps"]):
            losses.append(fb())
            trainer.optimizer.step()
        Fn.DIAG_SWITCHES.discard("bwd32path")
        Fn.DIAG_SWITCHES.discard("bwdf16")
    else:
      with Fn.precision(mode):
        trainer = Trainer(exp)
        model.zero_grad(set_to_none=True)
        out = model(batch)
        out.loss.backward()
        Fn.join_wgrad()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        del out
        model.zero_grad(set_to_none=True)
        losses = [float(trainer._eager_body(batch).metrics["ctc_loss"]) for _ in range(a["steps"])]
    torch.cuda.synchronize()
    Fn.set_deferred_wgrad([])
    del trainer, model, exp
    torch.cuda.empty_cache()
    Fn._FP32_BWD_ONLY.clear()
    for s in switches:
        Fn.DIAG_SWITCHES.discard(s)
    return grads, losses


def report(tag, g, gref, losses):
    acc = {}
    for n, r in gref.items():
        x = g.get(n, torch.zeros_like(r))
        d = acc.setdefault(kind_of(n), [0.0, 0.0, 0.0, 0.0, 0, 0])
        d[0] += float((x - r).double().norm() ** 2)
        d[1] += float(r.double().norm() ** 2)
        d[2] += float((r * torch.sign(x)).double().sum())
        d[3] += float(r.double().abs().sum())
        d[4] += int(((torch.sign(x) != torch.sign(r)) & (r != 0)).sum())
        d[5] += r.numel()
    tot = [sum(v[i] for k, v in acc.items() if k != "brain") for i in range(6)]
    acc["w2v_all"] = tot
    rel = [abs(x - y) / abs(y) for x, y in zip(losses, ref_losses)]
    parts = [f"{k} relL2 {(v[0] / max(v[1], 1e-300)) ** 0.5:.2e} eff {v[2] / max(v[3], 1e-300):.4f} "
             f"flip {v[4] / max(v[5], 1):.4f}" for k, v in sorted(acc.items())]
    print(f"[{name}] {tag}: loss rel vs reference {['%.2e' % r for r in rel]} ({['%.5f' % v for v in losses]})\n    "
          + "\n    ".join(parts), flush=True)


t0 = time.time()
gref, lref = run("fp32")
report("fp32 mode", gref, gref, lref)
print(f"  ({time.time() - t0:.1f} s)", flush=True)
for v in variants:
    t0 = time.time()
    bo, sw, em, mode = (), (), None, "bf16"
    if v.startswith("M:"):   # M:<mode>[/switch+switch]
        mode, _, xs = v[2:].partition("/")
        sw = tuple(filter(None, xs.split("+")))
    elif v.startswith("E:"):
        _, bw, sc = v.split(":")
        em = (bw, float(sc))
    elif v.startswith("B:"):
        bo = tuple(v[2:].split("+"))
    elif v.startswith("X:"):
        sw = tuple(v[2:].split("+"))
    g, l = run(mode, bo, sw, em)
    report(f"{mode} [{v}]", g, gref, l)
    print(f"  ({time.time() - t0:.1f} s)", flush=True)
