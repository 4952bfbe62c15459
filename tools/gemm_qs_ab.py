"""A/B of the quarter-scheduled operand DMA in the 256-column ping-pong GEMM (b2p_gemm16_variant 0) against
the 2-buffer schedule (variant 1) on the step's k-contiguous shapes and epilogues, interleaved rounds in one
process (guide §5.4 rule 24); outputs compared bitwise (same MFMA order).
usage: python tools/gemm_qs_ab.py [rounds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import build_lib  # noqa: E402

build_lib.ensure_built()
from wav2vec2forbrain_amd import functional as Fn, _lib  # noqa: E402

BF = torch.bfloat16
NT = 7968
# (M, N, K, epilogue, fp16 operands): the forward GEMMs the step runs on the 256-column kernel, the
# act'-backward, and square / odd shapes
SHAPES = [(NT, 3072, 768, "badhhB", True), (NT, 3072, 768, "gdhc", False), (NT, 4096, 1024, "badhhB", True),
          (NT, 4096, 1024, "gdhc", False), (NT, 3072, 1024, "bhh", True), (NT, 2304, 768, "bhh", True),
          (NT, 3072, 768, "f", False), (NT, 768, 3072, "f", False), (NT, 1024, 4096, "f", False),
          (4096, 4096, 4096, "f", False), (8192, 8192, 8192, "f", False), (8000, 3072, 776, "f", False)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lib = _lib.load()
    torch.manual_seed(0)
    os.environ.setdefault("B2P_GEMM16_PP", "2")
    for M, N, K, epi, h16 in SHAPES:
        dt = torch.float16 if h16 else BF
        a = torch.randn(M, K, device="cuda").to(dt)
        b = torch.randn(N, K, device="cuda").to(dt)
        A, B = Fn.op(a, 0, K, True), Fn.op(b, 0, K, True)
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(N, device="cuda")
        if "a" in epi:
            kw["act"] = Fn.ACT["gelu"]
            kw["pre16"] = torch.empty(M, N, device="cuda", dtype=BF)
        if "g" in epi:
            kw["act_bwd"] = Fn.ACT["gelu"]
            kw["aux16"] = torch.randn(M, N, device="cuda").to(BF)
        if "d" in epi:
            kw.update(drop_p=0.1, seed=7)
        if "h" in epi:
            kw["C16"] = torch.empty(M, N, device="cuda", dtype=BF)
            kw["c16_fp16"] = "hh" in epi
        if "B" in epi:   # the bf16 copy the FFN1 forward writes for its weight gradient
            kw["C16b"] = torch.empty(M, N, device="cuda", dtype=BF)
        if "c" in epi:
            kw["colsum_part"] = Fn.colsum_parts_buf(M, N, "cuda")
        C = torch.empty(M, N, device="cuda") if "f" in epi else None
        outs, times = {}, {0: [], 1: []}
        prec = "bf16"
        for r in range(rounds):
            for v in (0, 1):
                lib.b2p_gemm16_variant(v)
                fn = lambda: Fn.gemm(M, N, K, A, B, C, N, **kw)
                with Fn.precision(prec):
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
                outs[v] = [t.clone() for t in (C, kw.get("C16"), kw.get("pre16"), kw.get("C16b")) if t is not None]
        lib.b2p_gemm16_variant(0)
        same = all(torch.equal(x, y) for x, y in zip(outs[0], outs[1]))
        fl = 2.0 * M * N * K
        t0, t1 = sorted(times[0])[len(times[0]) // 2], sorted(times[1])[len(times[1]) // 2]
        print(f"{M}x{N}x{K} [{epi}{' f16' if h16 else ''}]  quarter {t0:8.1f} us {fl / t0 / 1e6:7.1f} TF   2-buffer {t1:8.1f} us "
              f"{fl / t1 / 1e6:7.1f} TF   q/2b {t0 / t1:5.3f}   bitwise {same}", flush=True)


if __name__ == "__main__":
    main()
