"""Per-step GRU kernels (csrc/gru.hip) at the Conformer encoder's shape: H=512, B=32, T'=249,
bidirectional, IN=512 (layers 1-2): fwd and bwd time per call (the host loop of T' launches)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from wav2vec2forbrain_amd import functional as Fn  # noqa: E402


def main():
    B, T, H, IN = 32, 249, 512, 512
    torch.manual_seed(0)
    ws = []
    for d in range(2):
        ws += [torch.randn(3 * H, IN, device="cuda") * 0.04, torch.randn(3 * H, H, device="cuda") * 0.04,
               torch.randn(3 * H, device="cuda") * 0.1, torch.randn(3 * H, device="cuda") * 0.1]
    ws = [w.requires_grad_(True) for w in ws]
    x = torch.randn(B, T, IN, device="cuda", requires_grad=True)
    dout = torch.randn(B, T, 2 * H, device="cuda")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with Fn.precision("bf16"):
        for it in range(4):
            s.record()
            out = Fn.gru_layer(x, H, 2, ws, None)
            e.record()
            torch.cuda.synchronize()
            tf = s.elapsed_time(e)
            s.record()
            torch.autograd.grad(out, [x] + ws, dout)
            e.record()
            torch.cuda.synchronize()
            tb = s.elapsed_time(e)
            print(f"gru H={H} B={B} T={T}: fwd {tf:.2f} ms, bwd {tb:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
