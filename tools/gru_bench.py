"""Times the bf16 persistent GRU kernels (b2p_gru_fwd16 / b2p_gru_bwd16) at the bench shape.
usage: python tools/gru_bench.py [B] [T] [H]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from wav2vec2forbrain_amd import _lib


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 249
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    nd = 2
    dev = "cuda"
    lnf = lambda R: int(_lib.load().b2p_gru16_lane_floats(B, T, H, nd, R))
    giL = torch.randn(lnf(3), device=dev)
    whh = torch.randn(nd, 3 * H, H, device=dev) / H ** 0.5
    bhh = torch.randn(nd, 3 * H, device=dev) * 0.1
    hL = torch.empty(lnf(1), device=dev)
    savL = torch.empty(lnf(4), device=dev)
    doL = torch.randn(lnf(1), device=dev)
    dgL = torch.empty(lnf(4), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    p = lambda t: t.data_ptr()

    def fwd():
        _lib.call("b2p_gru_fwd16", p(giL), p(whh), p(bhh), None, p(hL), p(savL), B, T, H, nd, st)

    def bwd():
        _lib.call("b2p_gru_bwd16", p(doL), p(whh), p(hL), p(savL), None, p(dgL), None, B, T, H, nd, st)

    for name, f in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 5
        e0.record()
        for _ in range(n):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f"{name} B={B} T={T} H={H} var={os.environ.get('B2P_GRU_VAR', '0')}: {ms * 1e3:.1f} us "
              f"({ms * 1e3 / T:.2f} us/step)", flush=True)


if __name__ == "__main__":
    main()
