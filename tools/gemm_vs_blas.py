"""Our bf16 GEMM (gemm16) vs torch.matmul (hipBLASLt) on the step's GEMM shapes: TFLOP/s per shape.
Both write fp32... torch writes bf16 (its native output), ours fp32 C; noted in the output."""
import os
import sys
import json

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import functional as Fn  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(5):
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
    NT, D, F = 7968, 768, 3072
    shapes = [("nt", NT, D, D), ("nt", NT, F, D), ("nt", NT, D, F), ("nt", NT, 3 * D, D),
              ("nn", NT, D, F), ("nn", NT, F, D), ("tn", D, F, NT), ("tn", F, D, NT), ("tn", D, D, NT),
              ("nt", 4096, 4096, 4096), ("nt", 8192, 8192, 8192)]
    # the Conformer-large step's shapes (D 1024, F 4096)
    Dc, Fc = 1024, 4096
    shapes += [("nt", NT, Fc, Dc), ("nt", NT, Dc, Fc), ("nt", NT, 3 * Dc, Dc), ("nt", NT, Dc, Dc), ("nn", NT, Dc, Fc),
               ("nn", NT, Fc, Dc), ("tn", Dc, Fc, NT), ("tn", Fc, Dc, NT), ("tn", Dc, Dc, NT)]
    if os.environ.get("GVB_SWEEP"):
        shapes = [("nt", 8192, 2048, k) for k in (256, 512, 1024, 2048, 4096, 8192)] + \
                 [("nt", 4096, 4096, k) for k in (768, 4096)] + [("nt", 7968, 3072, 768)]
    for kind, M, N, K in shapes:
        bf = torch.bfloat16
        if kind == "nt":
            a = torch.randn(M, K, device=dev, dtype=bf)
            w = torch.randn(N, K, device=dev, dtype=bf)
            ours = lambda: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), out, N)
            blas = lambda: torch.matmul(a, w.t())
        elif kind == "nn":
            a = torch.randn(M, K, device=dev, dtype=bf)
            w = torch.randn(K, N, device=dev, dtype=bf)
            ours = lambda: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, N, False), out, N)
            blas = lambda: torch.matmul(a, w)
        else:
            a = torch.randn(K, M, device=dev, dtype=bf)
            w = torch.randn(K, N, device=dev, dtype=bf)
            ours = lambda: Fn.gemm(M, N, K, Fn.op(a, 0, M, False), Fn.op(w, 0, N, False), out, N)
            blas = lambda: torch.matmul(a.t(), w)
        out = torch.empty(M, N, device=dev)
        o16 = torch.empty(M, N, device=dev, dtype=bf)
        fl = 2 * M * N * K
        t1 = timeit(ours)
        o_save = out
        out = None
        # the same launch writing only the bf16 copy (the byte count torch.matmul writes)
        t3 = timeit(lambda: _ours16(kind, M, N, K, a, w, o16))
        out = o_save
        t2 = timeit(blas)
        print(json.dumps(dict(shape=f"{kind} {M}x{N}x{K}", ours_us=round(t1 * 1e3, 1), ours_tf=round(fl / t1 / 1e9, 1),
                              ours16_us=round(t3 * 1e3, 1), ours16_tf=round(fl / t3 / 1e9, 1),
                              blas_us=round(t2 * 1e3, 1), blas_tf=round(fl / t2 / 1e9, 1))), flush=True)


def _ours16(kind, M, N, K, a, w, o16):
    if kind == "nt":
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), None, N, C16=o16)
    elif kind == "nn":
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, N, False), None, N, C16=o16)
    else:
        Fn.gemm(M, N, K, Fn.op(a, 0, M, False), Fn.op(w, 0, N, False), None, N, C16=o16)


if __name__ == "__main__":
    with Fn.precision("bf16"):
        main()
