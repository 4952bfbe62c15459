"""Times the fused bf16 attention kernels at the bench shape (B=32, T=249, 12 heads x 64).
usage: python tools/attn_bench.py [B] [T] [nh]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from wav2vec2forbrain_amd import functional as Fn


def timeit(f, n=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 249
nh = int(sys.argv[3]) if len(sys.argv) > 3 else 12
dh = 64
q = torch.randn(B * T, 3 * nh * dh, device="cuda") * 0.5
dO = torch.randn(B * T, nh * dh, device="cuda").to(torch.bfloat16)
fl = 4.0 * B * nh * T * T * dh
for kind in ("f16", "bf16"):
    for p in (0.0, 0.1):
        if kind == "f16":
            q16 = q.to(torch.float16)
            fwd = lambda: Fn._attn16_fwd_f16(q16, B, T, nh, dh, p, 5)
            _, _, lse2, mask = fwd()
        else:
            q16 = q.to(torch.bfloat16)
            fwd = lambda: Fn._attn16_fwd(q16, B, T, nh, dh, p, 5, want_mask=True)
            _, lse2, mask = fwd()
        tf = timeit(fwd)
        tb = timeit(lambda: Fn._attn16_bwd(q16, dO, lse2, B, T, nh, dh, p, 5, mask=mask))
        print(f"attn16[{kind}] B={B} T={T} nh={nh} p={p}: fwd {tf:.1f} us ({fl / tf / 1e6:.0f} TFLOP/s), "
              f"bwd {tb:.1f} us ({2.5 * fl / tb / 1e6:.0f} TFLOP/s)", flush=True)
# the bf16 mode's forward with the keep bits drawn ahead (functional.attn_keep_plan: b2p_attn16_keep_masks
# + b2p_attn16_fwd_f16_keep, DM 3), and the draw itself for one layer
import ctypes
q16 = q.to(torch.float16)
masks = torch.empty(1, B, nh, T, 8, device="cuda", dtype=torch.int32)
seeds = (ctypes.c_uint64 * 1)(5)
draw = lambda: Fn._lib.call("b2p_attn16_keep_masks", masks.data_ptr(), ctypes.addressof(seeds), 1, B, T, nh, 0.1, Fn._st())
draw()
Oh = torch.empty(B * T, nh * dh, device="cuda", dtype=torch.float16)
Ob = torch.empty(B * T, nh * dh, device="cuda", dtype=torch.bfloat16)
lse2 = torch.empty(B, nh, T, device="cuda")
fk = lambda: Fn._lib.call("b2p_attn16_fwd_f16_keep", q16.data_ptr(), Oh.data_ptr(), Ob.data_ptr(), lse2.data_ptr(), B, T,
                          nh, dh, float(dh ** -0.5), 0.1, masks[0].data_ptr(), Fn._st())
tf, td = timeit(fk), timeit(draw)
print(f"attn16[f16, keep bits read] B={B} T={T} nh={nh} p=0.1: fwd {tf:.1f} us ({fl / tf / 1e6:.0f} TFLOP/s); "
      f"keep-mask draw {td:.1f} us per layer", flush=True)
