"""One GEMM shape, repeated (for rocprofv3 --pmc passes): python tools/gemm_one.py nt 7968 3072 768 [iters]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import functional as Fn  # noqa: E402


def main():
    kind, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    b16 = len(sys.argv) > 6 and sys.argv[6] == "b16"
    cv = (lambda t: t.to(torch.bfloat16)) if b16 else (lambda t: t)
    torch.manual_seed(0)
    dev = "cuda"
    out = torch.empty(M, N, device=dev)
    if kind == "nt":
        a, b = cv(torch.randn(M, K, device=dev)), cv(torch.randn(N, K, device=dev))
        A, B = Fn.op(a, 0, K, True), Fn.op(b, 0, K, True)
    elif kind == "nn":
        a, b = cv(torch.randn(M, K, device=dev)), cv(torch.randn(K, N, device=dev))
        A, B = Fn.op(a, 0, K, True), Fn.op(b, 0, N, False)
    else:
        a, b = cv(torch.randn(K, M, device=dev)), cv(torch.randn(K, N, device=dev))
        A, B = Fn.op(a, 0, M, False), Fn.op(b, 0, N, False)
    with Fn.precision("bf16"):
        for _ in range(iters):
            Fn.gemm(M, N, K, A, B, out, N)
    torch.cuda.synchronize()
    ref = (a.double() if kind != "tn" else a.double().t()) @ (b.double().t() if kind == "nt" else b.double())
    err = ((out.double() - ref).norm() / ref.norm()).item()
    print(f"{kind} {M}x{N}x{K} {'b16' if b16 else 'f32'} rel_l2={err:.3e}")


if __name__ == "__main__":
    main()
