"""A/B of the narrow ping-pong GEMM (PBM x 128 tiles, b2p_gemm16_variant bit 2 clear) against the 128 x 128
kernel (bit 2 set) on the encoders' N <= 1024 shapes with their epilogues, interleaved rounds in one
process; outputs compared against each other (same K order inside a tile: bitwise) and timed.
usage: python tools/gemm_pn_ab.py [rounds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import build_lib  # noqa: E402

build_lib.ensure_built()
from wav2vec2forbrain_amd import functional as Fn, _lib  # noqa: E402

BF = torch.bfloat16
NT = 7968
# (M, N, K, epilogue, fp16 operands): r residual, f fp32 C, h bf16 C16, H fp16 C16, b bias, d dropout,
# c column sums
SHAPES = [(NT, 768, 3072, "rf", False), (NT, 768, 2304, "rf", False), (NT, 768, 768, "h", False),
          (NT, 768, 3072, "bdrf", True), (NT, 768, 768, "bdrf", True), (NT, 1024, 4096, "rf", False),
          (NT, 1024, 1024, "f", False), (NT, 1024, 2048, "f", False), (NT, 1024, 3072, "rf", False),
          (NT, 1024, 4096, "bdrf", True), (NT, 1024, 1024, "bdrf", True), (NT, 768, 768, "hc", False),
          (8000, 776, 1000, "f", False)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lib = _lib.load()
    torch.manual_seed(0)
    for M, N, K, epi, h16 in SHAPES:
        dt = torch.float16 if h16 else BF
        a = torch.randn(M, K, device="cuda").to(dt)
        b = torch.randn(N, K, device="cuda").to(dt)
        A, B = Fn.op(a, 0, K, True), Fn.op(b, 0, K, True)
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(N, device="cuda")
        if "d" in epi:
            kw.update(drop_p=0.1, seed=7)
        if "r" in epi:
            kw["residual"] = torch.randn(M, N, device="cuda")
        if "h" in epi or "H" in epi:
            kw["C16"] = torch.empty(M, N, device="cuda", dtype=BF)
            kw["c16_fp16"] = "H" in epi
        if "c" in epi:
            kw["colsum_part"] = Fn.colsum_parts_buf(M, N, "cuda")
        C = torch.empty(M, N, device="cuda") if "f" in epi else None
        outs, times = {}, {0: [], 2: []}
        for r in range(rounds):
            for v in (0, 2):
                lib.b2p_gemm16_variant(v)
                fn = lambda: Fn.gemm(M, N, K, A, B, C, N, **kw)
                with Fn.precision("bf16"):
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
                outs[v] = [t.clone() for t in (C, kw.get("C16"), kw.get("colsum_part")) if t is not None]
        lib.b2p_gemm16_variant(0)
        same = all(torch.equal(x, y) for x, y in zip(outs[0][:2], outs[2][:2]))
        err = max(float((x.float() - y.float()).norm() / (y.float().norm() + 1e-30)) for x, y in zip(outs[0], outs[2]))
        fl = 2.0 * M * N * K
        t0, t1 = sorted(times[0])[len(times[0]) // 2], sorted(times[2])[len(times[2]) // 2]
        print(f"{M}x{N}x{K} [{epi}{' f16' if h16 else ''}]  narrow {t0:7.1f} us {fl / t0 / 1e6:6.1f} TF   128x128 {t1:7.1f} us "
              f"{fl / t1 / 1e6:6.1f} TF   n/s {t0 / t1:5.3f}   bitwise {same} relerr {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
