"""GEMM epilogue cost on the FFN shapes (bf16 operands): the same GEMM with the step's epilogues.
python tools/epi_bench.py [M N K]  -> one JSON line per variant (us per launch, TF/s)."""
import json
import os
import sys

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
    return s.elapsed_time(e) / iters * 1e3


def main():
    M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (7968, 3072, 768)
    dev = "cuda"
    torch.manual_seed(0)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    c32 = torch.empty(M, N, device=dev)
    c16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    pre16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    aux16 = torch.randn(M, N, device=dev).to(torch.bfloat16)
    parts = Fn.colsum_parts_buf(M, N, dev)
    A, B = Fn.op(a, 0, K, True), Fn.op(w, 0, K, True)
    G = Fn.ACT["gelu"]
    variants = {
        "c16": lambda: Fn.gemm(M, N, K, A, B, None, N, C16=c16),
        "c32": lambda: Fn.gemm(M, N, K, A, B, c32, N),
        "bias_gelu_pre16_c16": lambda: Fn.gemm(M, N, K, A, B, None, N, bias=bias, act=G, pre16=pre16, C16=c16),
        "bias_gelu_drop_pre16_c16 (FFN1 fwd)": lambda: Fn.gemm(M, N, K, A, B, None, N, bias=bias, act=G, pre16=pre16,
                                                               drop_p=0.1, seed=5, C16=c16),
        "drop_gelu'_c16_colsum (FFN1 dgrad)": lambda: Fn.gemm(M, N, K, A, B, None, N, act_bwd=G, aux16=aux16,
                                                              drop_p=0.1, seed=5, C16=c16, colsum_part=parts),
        "gelu'_c16 (no dropout)": lambda: Fn.gemm(M, N, K, A, B, None, N, act_bwd=G, aux16=aux16, C16=c16),
    }
    for k, f in variants.items():
        us = timeit(f)
        print(json.dumps(dict(shape=f"{M}x{N}x{K}", epilogue=k, us=round(us, 2), tflops=round(2 * M * N * K / us / 1e6, 1))))


if __name__ == "__main__":
    with Fn.precision("bf16"):
        main()
