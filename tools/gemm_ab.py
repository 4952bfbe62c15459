"""GEMM A/B on the base step's encoder shapes (bf16 operands, the epilogues the step uses): mean launch
time and TF/s per shape under the current B2P_GEMM16_* environment. Run once per setting:
    B2P_GEMM16_TALL=0 python tools/gemm_ab.py ; B2P_GEMM16_TALL=1 python tools/gemm_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import build_lib  # noqa: E402

build_lib.ensure_built()
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def case(M, N, K, epi, a_k=True, b_k=True):
    dev = "cuda"
    a = torch.randn(M, K, device=dev).to(BF) if a_k else torch.randn(K, M, device=dev).to(BF)
    b = torch.randn(N, K, device=dev).to(BF) if b_k else torch.randn(K, N, device=dev).to(BF)
    A = Fn.op(a, 0, K if a_k else M, a_k)
    B = Fn.op(b, 0, K if b_k else N, b_k)
    kw = {}
    C = None
    if "f" in epi:
        C = torch.empty(M, N, device=dev)
    if "h" in epi:
        kw["C16"] = torch.empty(M, N, device=dev, dtype=BF)
    if "b" in epi:
        kw["bias"] = torch.randn(N, device=dev)
    if "a" in epi:
        kw["act"] = Fn.ACT["gelu"]
        kw["pre16"] = torch.empty(M, N, device=dev, dtype=BF)
    if "g" in epi:
        kw["act_bwd"] = Fn.ACT["gelu"]
        kw["aux16"] = torch.empty(M, N, device=dev, dtype=BF)
    if "d" in epi:
        kw["drop_p"] = 0.1
        kw["seed"] = 7
    if "r" in epi:
        kw["residual"] = torch.randn(M, N, device=dev)
    if "c" in epi:   # fused bias-gradient column sums
        kw["colsum_part"] = Fn.colsum_parts_buf(M, N, dev)
    fn = lambda: Fn.gemm(M, N, K, A, B, C, N, **kw)
    us = timeit(fn)
    tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
    return us, tf


SHAPES = [
    (7968, 3072, 768, "badh", True, True),    # FFN1 forward
    (7968, 3072, 768, "gdhc", True, True),    # FFN1 dgrad (GELU', dropout, bias-gradient column sums)
    (7968, 768, 3072, "bdrf", True, True),    # FFN2 forward
    (7968, 768, 3072, "rf", True, True),      # dx1
    (7968, 2304, 768, "bh", True, True),      # QKV
    (7968, 768, 2304, "rf", True, True),      # dx (QKV dgrad)
    (7968, 768, 768, "bdrf", True, True),     # out-projection
    (7968, 768, 768, "h", True, True),        # dO
    (3072, 768, 7968, "f", False, False),     # weight gradients (K = tokens, split-K)
    (768, 768, 7968, "f", False, False),
    (7968, 4096, 1024, "badh", True, True),   # Conformer-large FFN1 forward
    (7968, 1024, 4096, "bdrf", True, True),   # Conformer-large FFN2 forward
    (7968, 3072, 1024, "bh", True, True),     # Conformer-large QKV
    (7968, 2048, 1024, "bh", True, True),     # Conformer-large pointwise conv 1
    (4096, 1024, 7968, "f", False, False),    # Conformer-large FFN weight gradient
]

if __name__ == "__main__":
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("B2P_GEMM16"))
    tot = 0.0
    only = os.environ.get("GEMM_AB_ONLY")   # e.g. 3072x768x7968
    with Fn.precision("bf16"):
        for M, N, K, epi, ak, bk in SHAPES:
            if only and f"{M}x{N}x{K}" not in only.split(","):
                continue
            us, tf = case(M, N, K, epi, ak, bk)
            tot += us
            print(f"[{tag or 'default'}] {M}x{N}x{K} {epi:5s} {'A' if ak else 'a'}{'B' if bk else 'b'}: "
                  f"{us:8.1f} us {tf:7.1f} TF/s", flush=True)
    print(f"[{tag or 'default'}] total {tot:.1f} us", flush=True)
