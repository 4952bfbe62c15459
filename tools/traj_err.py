"""Attribution of the bf16-mode trajectory drift on a bench workload (VERDICT r3 "next" 1).

For each variant (blocks listed run forward AND backward in exact fp32: Fn._FP32_OPS with
Fn._BWD_FOLLOWS_FWD), against the exact-fp32 mode of the same model on the same batch:
  * the step-1 gradient of every brain_encoder.* parameter (the only gradients Adam consumes):
    relative L2 error, and the descent efficiency of a sign update (sum g_ref * sign(g) / sum |g_ref|,
    1.0 = Adam's first step goes exactly where the exact gradient points);
  * the CTC losses of `steps` deterministic Trainer steps (Adam lr 1e-3 over the brain encoder).
usage: python tools/traj_err.py [conformer|base] [steps] [variant,variant,...]
variants: names of Fn._FP32_OPS sets joined by '+', e.g. attn+ffn ; '-' = plain bf16; prefix F: = the
forward only (backward in bf16), except blocks marked *name (forward and backward); recur / recurfwd /
recurbwd = the GRU recurrence on the per-step fp32 kernels in both passes / the forward / the backward;
prefix B: = the blocks' backward only (Fn._FP32_BWD_ONLY), forward in the mode's precision."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from wav2vec2forbrain_amd import functional as Fn
from wav2vec2forbrain_amd.train.train_loop import Trainer
from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment, bench_config, build_model, device_batch

kind = sys.argv[1] if len(sys.argv) > 1 else "conformer"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
variants = (sys.argv[3] if len(sys.argv) > 3 else "-,attn,ffn,conv,gru,linear,front,attn+ffn+conv").split(",")
cfg = bench_config(kind)
dev = "cuda"
batch = device_batch(cfg, dev)
Fn._BWD_FOLLOWS_FWD[0] = True


RECUR = {"recur": (False, None), "recurfwd": (False, True), "recurbwd": (True, False)}


def run(mode, ops, fwd_only=False, bwd_only=()):
    Fn._BWD_FOLLOWS_FWD[0] = not fwd_only
    Fn._FP32_OPS.clear()
    Fn._FP32_OPS.update(o.lstrip("*") for o in ops if o not in RECUR)
    Fn._FP32_BWD_OPS.clear()
    Fn._FP32_BWD_OPS.update(o[1:] for o in ops if o.startswith("*"))
    Fn._FP32_BWD_ONLY.clear()
    Fn._FP32_BWD_ONLY.update(bwd_only)
    Fn._GRUMC[0], Fn._GRUMC_BWD[0] = True, None
    for o in ops:   # multi-CU GRU recurrence (bf16 MFMA) vs per-step fp32 kernels, per direction of the pass
        if o in RECUR:
            Fn._GRUMC[0], Fn._GRUMC_BWD[0] = RECUR[o]
    model = build_model(cfg, dev)
    model.train()
    for m in model.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = False
    with Fn.precision(mode):
        trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
        # step-1 gradient (before any update)
        model.zero_grad(set_to_none=True)
        out = model(batch)
        out.loss.backward()
        Fn.join_wgrad()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()
                 if n.startswith("brain_encoder.") and p.grad is not None}
        grads["<logits>"] = out.logits.detach().clone()
        del out
        losses = [float(trainer._eager_body(batch).metrics["ctc_loss"]) for _ in range(steps)]
    torch.cuda.synchronize()
    Fn.set_deferred_wgrad([])
    del trainer, model
    torch.cuda.empty_cache()
    Fn._FP32_OPS.clear()
    Fn._FP32_BWD_ONLY.clear()
    return grads, losses


t0 = time.time()
gref, lref = run("fp32", [])
lg_ref = gref.pop("<logits>")
print(f"[{kind}] fp32 mode losses {['%.6f' % v for v in lref]} ({time.time() - t0:.1f} s)", flush=True)
for v in variants:
    fo = v.startswith("F:")
    bo = v.startswith("B:")
    ops = [] if v in ("-", "F:-") else v[2 * (fo or bo):].split("+")
    t0 = time.time()
    g, l = run("bf16", [] if bo else ops, fo, ops if bo else ())
    lg = g.pop("<logits>")
    lerr = float((lg - lg_ref).double().norm() / lg_ref.double().norm())
    num = den = eff_n = eff_d = 0.0
    rows = []
    for n, r in gref.items():
        x = g.get(n, torch.zeros_like(r))
        e = float((x - r).double().norm() / (r.double().norm() + 1e-30))
        en = float((r * torch.sign(x)).double().sum())
        ed = float(r.double().abs().sum())
        num += float((x - r).double().norm() ** 2)
        den += float(r.double().norm() ** 2)
        eff_n += en
        eff_d += ed
        rows.append((e, en / max(ed, 1e-30), n))
    rows.sort(reverse=True)
    rel = [abs(a - b) / abs(b) for a, b in zip(l, lref)]
    print(f"[{kind}] bf16 fp32-blocks[{v}]: loss rel vs fp32 mode {['%.2e' % r for r in rel]}; logits relL2 {lerr:.2e}; "
          f"brain grad relL2 "
          f"{(num / den) ** 0.5:.3e}, sign-descent eff {eff_n / eff_d:.5f}; worst: "
          + "; ".join(f"{n.replace('brain_encoder.', '')} {e:.2e}/{ef:.4f}" for e, ef, n in rows[:4])
          + f" ({time.time() - t0:.1f} s)", flush=True)
