"""Debug: multi-CU GRU vs per-step fp32 kernels (relative errors per output) and run-to-run determinism."""
import math
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from wav2vec2forbrain_amd import _lib  # noqa: E402


def rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-12)), float((a - b).norm() / b.norm())


for (B, T, H) in [(32, 249, 512), (33, 57, 512), (32, 249, 384)]:
    nd = 2
    torch.manual_seed(0)
    gi = torch.randn(B, T, nd * 3 * H, device="cuda")
    whh = torch.randn(nd, 3 * H, H, device="cuda") / math.sqrt(H)
    bhh = torch.randn(nd, 3 * H, device="cuda") * 0.1
    dout = torch.randn(B, T, nd * H, device="cuda")

    def run(mc):
        out = torch.empty(B, T, nd * H, device="cuda")
        sv = torch.empty(B, T, nd, 4, H, device="cuda")
        dgi = torch.empty(B, T, nd * 3 * H, device="cuda")
        dgh = torch.empty_like(dgi)
        if mc:
            ws = torch.empty(int(_lib.load().b2p_gru_mc_workspace(B, H, nd)), device="cuda", dtype=torch.uint8)
            _lib.call("b2p_gru_fwd_mc", gi.data_ptr(), whh.data_ptr(), bhh.data_ptr(), None, out.data_ptr(),
                      sv.data_ptr(), ws.data_ptr(), B, T, H, nd, _lib.stream_ptr())
            _lib.call("b2p_gru_bwd_mc", dout.data_ptr(), whh.data_ptr(), out.data_ptr(), sv.data_ptr(), None,
                      dgi.data_ptr(), dgh.data_ptr(), None, ws.data_ptr(), B, T, H, nd, _lib.stream_ptr())
            torch.cuda.synchronize()
            HDR.append(ws[:8].view(torch.int32).tolist())
        else:
            buf = torch.empty(nd, B, H, device="cuda")
            _lib.call("b2p_gru_fwd", gi.data_ptr(), whh.data_ptr(), bhh.data_ptr(), None, out.data_ptr(),
                      sv.data_ptr(), B, T, H, nd, _lib.stream_ptr())
            _lib.call("b2p_gru_bwd", dout.data_ptr(), whh.data_ptr(), out.data_ptr(), sv.data_ptr(), None,
                      dgi.data_ptr(), dgh.data_ptr(), None, buf.data_ptr(), B, T, H, nd, _lib.stream_ptr())
        torch.cuda.synchronize()
        return out, sv, dgi, dgh

    HDR = []
    ref = run(False)
    a = run(True)
    b = run(True)
    hdr = HDR
    print(B, T, H, "vs fp32 (maxrel, l2rel):", [rel(x, y) for x, y in zip(a, ref)], "hdr", hdr,
          "deterministic:", [bool(torch.equal(x, y)) for x, y in zip(a, b)], flush=True)
