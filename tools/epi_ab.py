"""Epilogue ablation of the fused encoder GEMMs at the base workload (7968 tokens): the same K loop with
the epilogue's parts added one at a time (bias, activation with its stored pre-activation, dropout, the
16-bit copies, act' with its aux read, bias-gradient column sums), median launch time per variant.
usage: python tools/epi_ab.py [M N K] (default 7968 3072 768)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import build_lib  # noqa: E402

build_lib.ensure_built()
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402

BF = torch.bfloat16
# letters: f fp32 C, h 16-bit C16 (H: fp16), B second bf16 copy, b bias, a GELU (+ pre16), d dropout,
# g GELU' on aux16, c column sums, r residual, s SiLU (+ pre16)
VARIANTS = ["f", "h", "H", "bH", "bHB", "baH", "baHB", "bdH", "badH", "badHB", "gh", "gdh", "ghc", "gdhc", "rf", "bdrf"]
# s: SiLU (+ pre16) instead of GELU (the Conformer's FFN); B2P_EPI_VARIANTS=bH,bsH,... picks a subset
if os.environ.get("B2P_EPI_VARIANTS"):
    VARIANTS = os.environ["B2P_EPI_VARIANTS"].split(",")


def main():
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (7968, 3072, 768)
    torch.manual_seed(0)
    dev = "cuda"
    a = torch.randn(M, K, device=dev)
    b = torch.randn(N, K, device=dev)
    for v in VARIANTS:
        h16 = "H" in v or v.startswith("b")   # forward epilogues run on fp16 operands in the bf16 mode
        dt = torch.float16 if h16 else BF
        A, B = Fn.op(a.to(dt), 0, K, True), Fn.op(b.to(dt), 0, K, True)
        keep = (A, B)
        kw = {}
        C = torch.empty(M, N, device=dev) if "f" in v else None
        if "h" in v or "H" in v:
            kw["C16"] = torch.empty(M, N, device=dev, dtype=BF)
            kw["c16_fp16"] = "H" in v
        if "B" in v:
            kw["C16b"] = torch.empty(M, N, device=dev, dtype=BF)
        if "b" in v:
            kw["bias"] = torch.randn(N, device=dev)
        if "a" in v or "s" in v:
            kw["act"] = Fn.ACT["gelu" if "a" in v else "silu"]
            kw["pre16"] = torch.empty(M, N, device=dev, dtype=BF)
        if "d" in v:
            kw.update(drop_p=0.1, seed=7)
        if "g" in v:
            kw["act_bwd"] = Fn.ACT["gelu"]
            kw["aux16"] = torch.randn(M, N, device=dev).to(BF)
        if "c" in v:
            kw["colsum_part"] = Fn.colsum_parts_buf(M, N, dev)
        if "r" in v:
            kw["residual"] = torch.randn(M, N, device=dev)
        fn = lambda: Fn.gemm(M, N, K, A, B, C, N, **kw)
        ts = []
        for _ in range(5):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 10 * 1e3)
        t = sorted(ts)[2]
        print(f"{M}x{N}x{K} [{v:6s}] {'f16' if h16 else 'bf16'} {t:8.1f} us  {2.0 * M * N * K / t / 1e6:7.1f} TF", flush=True)
        del keep


if __name__ == "__main__":
    main()
