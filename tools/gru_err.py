"""GRU layer error vs the fp32 oracle (bf16 mode), persistent vs per-step recurrence.
usage: python tools/gru_err.py B L H [C]"""
import math
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle.b2p2t_oracle import gru_direction, unfold as unfold_ref
from wav2vec2forbrain_amd import functional as Fn

B, L, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
C = int(sys.argv[4]) if len(sys.argv) > 4 else 256
k, s = 32, 4
torch.manual_seed(5)
xsrc = torch.randn(B, L, C)
IN = C * k
ws = []
for d in range(2):
    ws += [torch.randn(3 * H, IN) / math.sqrt(IN), torch.randn(3 * H, H) / math.sqrt(H), torch.randn(3 * H) * 0.1,
           torch.randn(3 * H) * 0.1]
wr = [w.clone().requires_grad_(True) for w in ws]
xr = xsrc.clone().requires_grad_(True)
xin = unfold_ref(xr, k, s)
ref = torch.cat([gru_direction(xin, *wr[4 * d:4 * d + 4], None, d == 1) for d in range(2)], -1)
dout = torch.randn_like(ref)
refg = torch.autograd.grad(ref, [xr, *wr], dout)
rel = lambda a, b: float((a - b).norm() / b.norm())
for g16 in (0, 1):
    Fn._GRU16[0] = bool(g16)
    for mode in ("bf16", "fp32"):
        with Fn.precision(mode):
            wg = [w.cuda().requires_grad_(True) for w in ws]
            xs = xsrc.cuda().requires_grad_(True)
            out = Fn.gru_layer(Fn.Unfolded(xs, k, s), H, 2, wg)
            got = torch.autograd.grad(out, [xs, *wg], dout.cuda())
        errs = [rel(a.cpu(), b) for a, b in zip(got, refg)]
        mean_shift = float((out.detach().cpu() - ref.detach()).mean())
        print(f"B={B} L={L} H={H} GRU16={g16} {mode}: out relL2 {rel(out.detach().cpu(), ref.detach()):.2e} "
              f"mean shift {mean_shift:.2e}; grads relL2 x {errs[0]:.2e} w_ih {errs[1]:.2e} w_hh {errs[2]:.2e} "
              f"b_ih {errs[3]:.2e} b_hh {errs[4]:.2e} | rev w_hh {errs[6]:.2e}", flush=True)
