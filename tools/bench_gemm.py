"""GEMM microbenchmark on the shapes of the base bs=32 L=1024 training step (TFLOP/s per shape)."""
import os
import sys
import json

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
    return s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    dev = "cuda"
    NT, D, F, T, B, nh = 7968, 768, 3072, 249, 32, 12
    res = []

    cv = (lambda t: t.to(torch.bfloat16)) if B16 else (lambda t: t)

    def lin(M, N, K, kind):
        a = cv(torch.randn(M, K, device=dev))
        w = cv(torch.randn(N, K, device=dev))
        out = torch.empty(M, N, device=dev)
        if kind == "nt":
            f = lambda: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), out, N)
        elif kind == "nn":
            bm = cv(torch.randn(K, N, device=dev))
            f = lambda: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(bm, 0, N, False), out, N)
        else:
            at = cv(torch.randn(K, M, device=dev))
            bm = cv(torch.randn(K, N, device=dev))
            f = lambda: Fn.gemm(M, N, K, Fn.op(at, 0, M, False), Fn.op(bm, 0, N, False), out, N)
        ms = timeit(f)
        res.append(dict(shape=f"{kind} {M}x{N}x{K}", ms=round(ms, 4), tflops=round(2 * M * N * K / ms / 1e9, 1)))

    for kind in ("nt", "nn", "tn"):
        lin(NT, D, D, kind)
        lin(NT, F, D, kind)
        lin(NT, D, F, kind)
    lin(D, F, NT, "tn")
    lin(4096, 4096, 4096, "nt")
    # GRU layer-0 implicit unfold projection
    L, C = 1024, 256
    x = cv(torch.randn(B, L, C, device=dev))
    wp = cv(torch.randn(1536, 8192, device=dev))
    gi = torch.empty(B * T, 1536, device=dev)
    A = Fn.conv_op(x, 0, C, T, L, 4, 0, C, L * C, True)
    ms = timeit(lambda: Fn.gemm(B * T, 1536, 8192, A, Fn.op(wp, 0, 8192, True), gi, 1536))
    res.append(dict(shape="unfold-proj 7968x1536x8192", ms=round(ms, 4), tflops=round(2 * B * T * 1536 * 8192 / ms / 1e9, 1)))
    if B16:
        for r in res:
            r["operands"] = "bf16"
        for r in res:
            print(json.dumps(r))
        return
    # pos-conv grouped
    e = torch.randn(B, T, D, device=dev)
    wq = torch.randn(D, 128 * 48, device=dev)
    o = torch.empty(B, T, D, device=dev)
    A = Fn.conv_op(e, 0, D, T, T, 1, 64, 48, T * D, True, bs1=48)
    ms = timeit(lambda: Fn.gemm(B * T, 48, 6144, A, Fn.op(wq, 0, 6144, True, bs1=48 * 6144), o, D, cbs1=48, nz1=16))
    res.append(dict(shape="posconv 16x(7968x48x6144)", ms=round(ms, 4), tflops=round(2 * B * T * 768 * 6144 / ms / 1e9, 1)))
    # attention batched
    Tp = 252
    qkv = torch.randn(NT, 3 * D, device=dev)
    S = torch.empty(B, nh, T, Tp, device=dev)
    ms = timeit(lambda: Fn.gemm(T, T, 64, Fn.op(qkv, 0, 3 * D, True, bs1=T * 3 * D, bs2=64),
                                Fn.op(qkv, D, 3 * D, True, bs1=T * 3 * D, bs2=64), S, Tp, cbs1=nh * T * Tp,
                                cbs2=T * Tp, nz1=B, nz2=nh))
    res.append(dict(shape="attn QK^T 384x(249x249x64)", ms=round(ms, 4), tflops=round(2 * 384 * T * T * 64 / ms / 1e9, 1)))
    O = torch.empty(NT, D, device=dev)
    ms = timeit(lambda: Fn.gemm(T, 64, T, Fn.op(S, 0, Tp, True, bs1=nh * T * Tp, bs2=T * Tp),
                                Fn.op(qkv, 2 * D, 3 * D, False, bs1=T * 3 * D, bs2=64), O, D, cbs1=T * D, cbs2=64,
                                nz1=B, nz2=nh))
    res.append(dict(shape="attn PV 384x(249x64x249)", ms=round(ms, 4), tflops=round(2 * 384 * T * T * 64 / ms / 1e9, 1)))
    for r in res:
        print(json.dumps(r))


B16 = False

if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    if mode == "b16":
        B16, mode = True, "bf16"
    with Fn.precision(mode):
        main()
