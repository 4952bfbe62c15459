"""The step's plain 16-bit GEMM shapes on the hipBLASLt path (b2p_gemm -> csrc/blaslt.cpp) against the
hand-written gemm16 kernels, in the epilogue form the step uses (fp32 out + residual, 16-bit out, fp32
out). usage: python tools/blaslt_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import functional as Fn  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


NT = 7968
shapes = [(NT, 768, 3072, "res"), (NT, 768, 2304, "res"), (NT, 768, 768, "c16"), (NT, 1024, 4096, "res"),
          (NT, 1024, 2048, "res"), (NT, 1024, 1024, "f32"), (NT, 1024, 1024, "c16"), (NT, 2048, 1024, "f32"),
          (NT, 256, 768, "f32")]
for M, N, K, form in shapes:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda") if form != "c16" else None
    C16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if form == "c16" else None
    res = torch.randn(M, N, device="cuda") if form == "res" else None
    f = lambda: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), C, N, residual=res, C16=C16)
    out = []
    for lib in (False, True):
        Fn.blaslt(lib)
        out.append(timeit(f))
    Fn.blaslt(True)
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K} {form:4s}  gemm16 {out[0]:7.1f} us ({fl / out[0] / 1e6:6.0f} TF)   hipBLASLt {out[1]:7.1f} us "
          f"({fl / out[1] / 1e6:6.0f} TF)", flush=True)
