"""Plain 16-bit GEMMs through hipBLASLt (csrc/blaslt.cpp) against the hand-written gemm16 kernels on the
same operands: every form the library path takes (k- / n-contiguous B, fp32 / bf16 / fp16 output, alpha,
beta accumulation, an added residual), launches counted, graph capture of planned shapes, and the forms it
must leave to the hand-written kernels (fused epilogues, weight-gradient layouts, batched launches)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fn():
    from wav2vec2forbrain_amd import functional as Fn
    return Fn


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def _run(Fn, lib, M, N, K, bk, dt, out, alpha=1.0, beta=0.0, residual=None, c0=None):
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda").to(dt)
    w = (torch.randn(N, K, device="cuda") if bk else torch.randn(K, N, device="cuda")).to(dt)
    Bop = Fn.op(w, 0, K, True) if bk else Fn.op(w, 0, N, False)
    C = C16 = None
    if out == "f32":
        C = torch.zeros(M, N, device="cuda") if c0 is None else c0.clone()
    else:
        C16 = torch.empty(M, N, device="cuda", dtype=torch.float16 if out == "f16" else torch.bfloat16)
    Fn.blaslt(lib)
    try:
        n0 = Fn._lib.load().b2p_blaslt_calls(1)
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Bop, C, N, alpha=alpha, beta=beta, residual=residual, C16=C16,
                c16_fp16=out == "f16")
        torch.cuda.synchronize()
        calls = Fn._lib.load().b2p_blaslt_calls(1)
    finally:
        Fn.blaslt(True)
    assert n0 >= 0
    ref = alpha * (a.float() @ (w.float().t() if bk else w.float()))
    if residual is not None:
        ref = ref + residual
    if c0 is not None and beta != 0.0:
        ref = ref + beta * c0
    return (C if C is not None else C16), ref, calls


@pytest.mark.parametrize("M,N,K", [(7968, 768, 3072), (7968, 1024, 1024), (300, 192, 256)])
@pytest.mark.parametrize("bk", [True, False])
@pytest.mark.parametrize("form", ["f32", "bf16", "f16", "residual", "beta"])
def test_blaslt_plain_gemm_matches_hand_written(M, N, K, bk, form):
    Fn = _fn()
    dt = torch.float16 if form == "f16" else torch.bfloat16
    out = form if form in ("bf16", "f16") else "f32"
    kw = {}
    if form == "residual":
        kw["residual"] = torch.randn(M, N, device="cuda")
    if form == "beta":
        kw["beta"], kw["c0"] = 1.0, torch.randn(M, N, device="cuda")
    kw["alpha"] = 0.5 if form == "f32" else 1.0
    got, ref, calls = _run(Fn, True, M, N, K, bk, dt, out, **kw)
    own, _, calls_own = _run(Fn, False, M, N, K, bk, dt, out, **kw)
    assert calls == 1 and calls_own == 0
    tol = 1e-5 if out == "f32" else 8e-3
    assert _rel(got, ref) < tol and _rel(own, ref) < tol, (_rel(got, ref), _rel(own, ref))
    assert _rel(got, own) < tol


def test_blaslt_leaves_fused_and_wgrad_gemms_to_gemm16():
    Fn = _fn()
    M, N, K = 512, 256, 384
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda")
    bias = torch.randn(N, device="cuda")
    lib = Fn._lib.load()
    lib.b2p_blaslt_calls(1)
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), C, N, bias=bias)            # fused bias
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), C, N, act=Fn.ACT["gelu"])  # fused act
    at = torch.randn(K, M, device="cuda").bfloat16()   # weight-gradient layout: A m-, B n-contiguous
    wt = torch.randn(K, N, device="cuda").bfloat16()
    Fn.gemm(M, N, K, Fn.op(at, 0, M, False), Fn.op(wt, 0, N, False), C, N)
    C16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), C, N, C16=C16)   # two outputs
    torch.cuda.synchronize()
    assert lib.b2p_blaslt_calls(1) == 0


def test_blaslt_graph_capture_replays_planned_shape():
    """A shape planned in an eager launch is captured into a graph and replays to the eager result;
    an unplanned shape met inside a capture runs on the hand-written kernel."""
    Fn = _fn()
    M, N, K = 2048, 768, 3072
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    res = torch.randn(M, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    lib = Fn._lib.load()
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), C, N, residual=res)
    torch.cuda.synchronize()
    eager = C.clone()
    a2 = torch.randn(640, 704, device="cuda").bfloat16()
    w2 = torch.randn(320, 704, device="cuda").bfloat16()
    C2 = torch.empty(640, 320, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    lib.b2p_blaslt_calls(1)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), C, N, residual=res)
            Fn.gemm(640, 320, 704, Fn.op(a2, 0, 704, True), Fn.op(w2, 0, 704, True), C2, 320)
    assert lib.b2p_blaslt_calls(1) == 1   # the planned shape only
    C.zero_()
    C2.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(C, eager)
    ref2 = a2.float() @ w2.float().t()
    assert _rel(C2, ref2) < 1e-5
    del g
