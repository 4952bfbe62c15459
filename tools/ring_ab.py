"""A/B of the 256-column GEMM kernels (b2p_gemm16_variant: 0 = the 2-buffer 64-deep ping-pong kernel, 1 =
the 5-slot ring kernel) on the step's shapes, in one process with interleaved rounds (guide §5.4 rule
24). With B2P_GEMM16_PP=2 every shape is forced onto the 256-column family; the two variants' outputs are
compared bitwise (same MFMA accumulation order).
usage: B2P_GEMM16_PP=2 python tools/ring_ab.py [rounds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import build_lib  # noqa: E402

build_lib.ensure_built()
from wav2vec2forbrain_amd import functional as Fn, _lib  # noqa: E402

BF = torch.bfloat16
NT, D, F, Dc, Fc = 7968, 768, 3072, 1024, 4096
# (kind, M, N, K, epilogue): nt = forward (A, B k-contiguous), nn = backward data ([K][N] weight),
# tn = weight gradient (both m/n-contiguous, K = tokens)
SHAPES = [("nt", NT, F, D, "f"), ("nt", NT, D, F, "f"), ("nt", NT, 3 * D, D, "f"), ("nt", NT, D, D, "f"),
          ("nt", NT, Fc, Dc, "f"), ("nt", NT, Dc, Fc, "f"), ("nt", NT, 3 * Dc, Dc, "f"), ("nt", NT, Dc, Dc, "f"),
          ("nn", NT, D, F, "f"), ("nn", NT, Fc, Dc, "f"),
          ("tn", D, F, NT, "f"), ("tn", Fc, Dc, NT, "f"), ("tn", Dc, Dc, NT, "f"),
          ("tn", F, D, NT, "f"), ("tn", D, D, NT, "f"), ("tn", 4096, 4096, 7968, "f"),
          ("nt", 4096, 4096, 4096, "f"), ("nt", 8192, 8192, 8192, "f"), ("nt", NT, F, D, "bdrh"), ("nt", 8000, 3072, 776, "f"),
          ("tn", 1000, 3000, 1000, "f")]


def operands(kind, M, N, K, dev="cuda"):
    if kind == "nt":
        a = torch.randn(M, K, device=dev).to(BF)
        b = torch.randn(N, K, device=dev).to(BF)
        return a, b, Fn.op(a, 0, K, True), Fn.op(b, 0, K, True)
    if kind == "nn":
        a = torch.randn(M, K, device=dev).to(BF)
        b = torch.randn(K, N, device=dev).to(BF)
        return a, b, Fn.op(a, 0, K, True), Fn.op(b, 0, N, False)
    a = torch.randn(K, M, device=dev).to(BF)
    b = torch.randn(K, N, device=dev).to(BF)
    return a, b, Fn.op(a, 0, M, False), Fn.op(b, 0, N, False)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lib = _lib.load()
    torch.manual_seed(0)
    with Fn.precision("bf16"):
        for kind, M, N, K, epi in SHAPES:
            a, b, A, B = operands(kind, M, N, K)
            kw = {}
            if "b" in epi:
                kw["bias"] = torch.randn(N, device="cuda")
            if "d" in epi:
                kw.update(drop_p=0.1, seed=7)
            if "r" in epi:
                kw["residual"] = torch.randn(M, N, device="cuda")
            if "h" in epi:
                kw["C16"] = torch.empty(M, N, device="cuda", dtype=BF)
            outs = {}
            times = {0: [], 1: []}
            for r in range(rounds):
                for v in (0, 1):
                    lib.b2p_gemm16_variant(v)
                    C = torch.empty(M, N, device="cuda")
                    fn = lambda: Fn.gemm(M, N, K, A, B, C, N, **kw)
                    for _ in range(2):
                        fn()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(10):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    times[v].append(s.elapsed_time(e) / 10 * 1e3)
                    outs[v] = (C.clone(), kw["C16"].clone() if "C16" in kw else None)
            lib.b2p_gemm16_variant(0)
            same = torch.equal(outs[0][0], outs[1][0]) and (outs[0][1] is None or torch.equal(outs[0][1], outs[1][1]))
            ref = None
            if not same:   # not bitwise: how far from an fp32 reference
                af, bf = a.float(), b.float()
                ref = (af @ bf.t() if kind == "nt" else af @ bf if kind == "nn" else af.t() @ bf)
            fl = 2.0 * M * N * K
            t0, t1 = sorted(times[0])[len(times[0]) // 2], sorted(times[1])[len(times[1]) // 2]
            msg = (f"{kind} {M}x{N}x{K} [{epi}]  pp {t0:8.1f} us {fl / t0 / 1e6:7.1f} TF   p4 {t1:8.1f} us "
                   f"{fl / t1 / 1e6:7.1f} TF   ring/pp {t1 / t0:5.3f}   bitwise {same}")
            if ref is not None and "b" not in epi:
                for v in (0, 1):
                    msg += f"  relerr[{v}] {float((outs[v][0] - ref).norm() / ref.norm()):.2e}"
            print(msg, flush=True)


if __name__ == "__main__":
    main()
