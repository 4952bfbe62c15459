"""GEMM kernel (b2p_gemm) against plain PyTorch fp32 references: layouts, tails, batching,
implicit conv/unfold views, epilogues, both MFMA precisions."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = {"fp32": (2e-5, 2e-5), "bf16": (2e-2, 2e-2), "bf16x3": (1e-4, 1e-4)}


def _fn():
    from wav2vec2forbrain_amd import functional as Fn
    return Fn


def _close(out, ref, mode, scale=None):
    rtol, atol = TOL[mode]
    scale = scale if scale is not None else ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= atol * scale + rtol * 0, f"max err {err} vs scale {scale} ({mode})"


@pytest.mark.parametrize("mode", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (130, 70, 37), (1, 33, 5), (300, 257, 96), (64, 48, 6144)])
def test_nt_nn_tn(mode, M, N, K):
    Fn = _fn()
    torch.manual_seed(0)
    Kp = (K + 3) // 4 * 4
    Np = (N + 3) // 4 * 4
    Mp = (M + 3) // 4 * 4
    a = torch.randn(M, Kp, device="cuda")
    w = torch.randn(N, Kp, device="cuda")
    with Fn.precision(mode):
        # NT: out = a[:, :K] @ w[:, :K]^T
        out = torch.empty(M, Np, device="cuda")
        Fn.gemm(M, N, K, Fn.op(a, 0, Kp, True), Fn.op(w, 0, Kp, True), out, Np)
        _close(out[:, :N], a[:, :K] @ w[:, :K].t(), mode)
        # NN: out = a[:, :K] @ b (b: K x N, row-major, ld Np)
        b = torch.randn(K, Np, device="cuda")
        out2 = torch.empty(M, Np, device="cuda")
        Fn.gemm(M, N, K, Fn.op(a, 0, Kp, True), Fn.op(b, 0, Np, False), out2, Np)
        _close(out2[:, :N], a[:, :K] @ b[:, :N], mode)
        # TN: out = at^T @ b with at: K x M (ld Mp)
        at = torch.randn(K, Mp, device="cuda")
        out3 = torch.empty(M, Np, device="cuda")
        Fn.gemm(M, N, K, Fn.op(at, 0, Mp, False), Fn.op(b, 0, Np, False), out3, Np)
        _close(out3[:, :N], at[:, :M].t() @ b[:, :N], mode)


@pytest.mark.parametrize("form", ["kernel", "image"])
@pytest.mark.parametrize("layout", ["nt", "tn"])
def test_split_bf16_accuracy(form, layout, monkeypatch):
    """precision 3 (split bf16, the bf16x3 mode): the relative error of a K = 4096 product against an fp64
    reference is within a few 2^-16 (the bf16 mode's is ~2^-9); K >= 2048 on 4 output tiles makes it a
    split-K launch (slabs summed in slice order); operands span 1e-6 .. 1e2 (bf16 keeps fp32's range).
    form kernel: the fp32-operand kernel's three MFMAs per k-step (csrc/gemm.hip precision 3); image: the
    split-bf16 operand images (b2p_split3_bf16) over K' = 3K on the bf16 LDS-DMA kernels."""
    Fn = _fn()
    monkeypatch.setattr(Fn, "_AUTO16_MIN_FLOP", 0.0 if form == "image" else 1e30)
    monkeypatch.setattr(Fn, "_X3_SPLIT", [form == "image"])
    torch.manual_seed(3)
    M, N, K = 256, 192, 4096
    a = torch.randn(M, K, device="cuda") * torch.logspace(-6, 2, K, device="cuda")[torch.randperm(K, device="cuda")]
    w = torch.randn(N, K, device="cuda")
    ref = a.double() @ w.double().t()
    at, wt = a.t().contiguous(), w.t().contiguous()   # K x M, K x N: the weight-gradient layout
    errs = {}
    for mode in ("bf16", "bf16x3"):
        with Fn.precision(mode):
            out = torch.empty(M, N, device="cuda")
            if layout == "nt":
                Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), out, N)
            else:
                Fn.gemm(M, N, K, Fn.op(at, 0, M, False), Fn.op(wt, 0, N, False), out, N)
        errs[mode] = float((out.double() - ref).norm() / ref.norm())
    print(errs)
    assert errs["bf16x3"] <= 3e-5, errs
    assert errs["bf16x3"] * 50 <= errs["bf16"], errs


@pytest.mark.parametrize("mode", ["fp32", "bf16", "bf16x3", "bf16x3-image"])
def test_epilogue(mode, monkeypatch):
    Fn = _fn()
    if mode == "bf16x3-image":   # the split-bf16 operand images on the bf16 kernels, every epilogue
        mode = "bf16x3"
        monkeypatch.setattr(Fn, "_AUTO16_MIN_FLOP", 0.0)
    torch.manual_seed(1)
    M, N, K = 200, 96, 64
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / 8
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    with Fn.precision(mode):
        out = torch.empty(M, N, device="cuda")
        pre = torch.empty(M, N, device="cuda")
        Fn.mm_nt(x, w, out, bias=bias, act=Fn.ACT["gelu"], pre_out=pre, residual=res)
        ref_pre = x @ w.t() + bias
        _close(pre, ref_pre, mode)
        _close(out, F.gelu(ref_pre) + res, mode, scale=ref_pre.abs().max().item())
        # beta accumulate + alpha
        c = torch.randn(M, N, device="cuda")
        c0 = c.clone()
        Fn.gemm(M, N, K, Fn.op(x, 0, K, True), Fn.op(w, 0, K, True), c, N, alpha=0.5, beta=2.0)
        _close(c, 0.5 * (x @ w.t()) + 2.0 * c0, mode, scale=ref_pre.abs().max().item() * 2)
        # act_bwd: out = acc * gelu'(aux)
        g = torch.empty(M, N, device="cuda")
        Fn.gemm(M, N, K, Fn.op(x, 0, K, True), Fn.op(w, 0, K, True), g, N, act_bwd=Fn.ACT["gelu"], aux=ref_pre)
        pr = ref_pre.clone().requires_grad_(True)
        (gg,) = torch.autograd.grad(F.gelu(pr), pr, x @ w.t())
        _close(g, gg, mode, scale=ref_pre.abs().max().item())


def test_dropout_epilogue_mask_consistent():
    Fn = _fn()
    M, N, K = 256, 128, 32
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    with Fn.precision("fp32"):
        out = torch.empty(M, N, device="cuda")
        Fn.gemm(M, N, K, Fn.op(x, 0, K, True), Fn.op(w, 0, K, True), out, N, drop_p=0.25, seed=1234)
        ref = x @ w.t()
        kept = out != 0
        frac = kept.float().mean().item()
        assert 0.72 < frac < 0.78
        torch.testing.assert_close(out[kept], ref[kept] / 0.75, rtol=1e-4, atol=1e-4)
        # same (seed, index) mask from the elementwise dropout kernel
        y = Fn._dropout_raw(torch.ones(M, N, device="cuda"), 0.25, 1234)
        assert torch.equal(y != 0, kept)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_batched_attention_layout(mode):
    Fn = _fn()
    torch.manual_seed(2)
    B, T, nh, dh = 3, 37, 4, 16
    D = nh * dh
    Tp = (T + 3) // 4 * 4
    qkv = torch.randn(B * T, 3 * D, device="cuda")
    S = torch.zeros(B, nh, T, Tp, device="cuda")
    with Fn.precision(mode):
        Fn.gemm(T, T, dh, Fn.op(qkv, 0, 3 * D, True, bs1=T * 3 * D, bs2=dh),
                Fn.op(qkv, D, 3 * D, True, bs1=T * 3 * D, bs2=dh), S, Tp, cbs1=nh * T * Tp, cbs2=T * Tp, nz1=B,
                nz2=nh, alpha=0.25)
    q = qkv.view(B, T, 3, nh, dh)[:, :, 0].transpose(1, 2)
    k = qkv.view(B, T, 3, nh, dh)[:, :, 1].transpose(1, 2)
    _close(S[..., :T], 0.25 * q @ k.transpose(-1, -2), mode)


def test_gather_batch_and_bias():
    """day-linear: per-sample B operand and bias selected through day_idxs."""
    Fn = _fn()
    torch.manual_seed(3)
    B, L, C, nd = 4, 40, 32, 6
    xs = torch.randn(B, L, C, device="cuda")
    W = torch.randn(nd, C, C, device="cuda")
    bias = torch.randn(nd, 1, C, device="cuda")
    day = torch.tensor([5, 0, 5, 2], device="cuda")
    out = torch.empty(B, L, C, device="cuda")
    with Fn.precision("fp32"):
        Fn.gemm(L, C, C, Fn.op(xs, 0, C, True, bs1=L * C), Fn.op(W, 0, C, False, bs1=C * C, gather=day), out, C,
                cbs1=L * C, nz1=B, bias=bias, biasbs1=C, bias_gather=day)
    ref = torch.einsum("btd,bdk->btk", xs, W[day]) + bias[day]
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_implicit_unfold_views(mode):
    """nn.Unfold((k,1), stride) + projection as one implicit GEMM, and its transposed use (dW)."""
    Fn = _fn()
    from oracle.b2p2t_oracle import unfold
    torch.manual_seed(4)
    B, L, C, k, s, N = 3, 72, 16, 8, 4, 40
    T = (L - k) // s + 1
    x = torch.randn(B, L, C, device="cuda")
    w = torch.randn(N, C * k, device="cuda")            # reference layout: col = c*k + tap
    u = unfold(x.cpu(), k, s).cuda()                     # (B, T, C*k)
    wp = torch.empty(N, k * C, device="cuda")
    Fn._lib.call("b2p_conv_weight_permute", w.data_ptr(), wp.data_ptr(), N, C, k, 0, Fn._st())
    with Fn.precision(mode):
        out = torch.empty(B * T, N, device="cuda")
        A = Fn.conv_op(x, 0, C, T, L, s, 0, C, L * C, True)
        Fn.gemm(B * T, N, k * C, A, Fn.op(wp, 0, k * C, True), out, N)
        _close(out, (u.view(B * T, -1) @ w.t()), mode)
        # dW' = dy^T @ unfold(x) (conv view as B operand, inner = n)
        dy = torch.randn(B * T, N, device="cuda")
        dwp = torch.empty(N, k * C, device="cuda")
        Bop = Fn.conv_op(x, 0, C, T, L, s, 0, C, L * C, False)
        Fn.gemm(N, k * C, B * T, Fn.op(dy, 0, N, False), Bop, dwp, k * C)
        dw = torch.empty(N, C * k, device="cuda")
        Fn._lib.call("b2p_conv_weight_permute", dwp.data_ptr(), dw.data_ptr(), N, C, k, 1, Fn._st())
        _close(dw, dy.t() @ u.view(B * T, -1), mode)


def test_bf16x3_role_forms():
    """The bf16x3 mode's per-role GEMM forms (functional._x3_form) on a backward-data layout (A k-contiguous,
    B n-contiguous): three-term split images (~16 bits per product), the two-term images of
    b2p_split3_bf16's pattern | 16 (one operand ~16 bits, the other bf16) and single-pass bf16, against an
    fp64 product: the error grows as terms are dropped, and the two-term forms sit between. (GEMMs under
    2 GFLOP keep the fp32-operand kernel's three-MFMA form whatever the role's form: this one is 4.3.)"""
    Fn = _fn()
    torch.manual_seed(12)
    M, N, K = 2048, 1024, 1024
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    ref = (a.double() @ b.double())

    def run(forms):
        out = torch.empty(M, N, device="cuda")
        with Fn.precision("bf16x3"), Fn.x3_forms(forms):
            Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(b, 0, N, False), out, N)
        return float(((out.double() - ref).norm() / ref.norm()).item())
    e3, e2a, e2b, e1 = run(()), run(("dgrad2a",)), run(("dgrad2b",)), run(("dgrad1",))
    print("bf16x3 role forms relL2: three-term", e3, "2a", e2a, "2b", e2b, "single", e1)
    assert e3 < 2e-5, e3
    assert e3 < e2a < e1 and e3 < e2b < e1, (e3, e2a, e2b, e1)
    assert e1 > 1e-3, e1


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
@pytest.mark.parametrize("M,N", [(7968, 32), (1000, 48), (20000, 32)])
def test_narrow_n_fp32_operands(mode, M, N):
    """fp32-operand GEMMs with N <= 64 (the CTC lm_head, 768 -> 32 classes): 64 x 64 tiles when the 128-row
    grid leaves most CUs idle, 128 x 64 otherwise; both against torch fp32, with the head's bias epilogue."""
    Fn = _fn()
    torch.manual_seed(9)
    K = 768
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / 16
    bias = torch.randn(N, device="cuda")
    with Fn.precision(mode):
        out = torch.empty(M, N, device="cuda")
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), out, N, bias=bias)
    _close(out, a @ w.t() + bias, mode)


@pytest.mark.parametrize("O,I,K", [(768, 256, 32), (1536, 256, 32), (3, 64, 64), (5, 4, 1024), (40, 16, 8),
                                    (768, 48, 128), (6, 12, 5)])
def test_conv_weight_permute_exact(O, I, K):
    """b2p_conv_weight_permute (the tap-major GRU input / pos-conv weight copies and their gradients'
    inverse) equals the torch permutation element for element, both directions: the 16-byte power-of-two
    form (I, K powers of two; the base / Conformer GRU weights, square and one-channel-wide shapes) and
    the scalar tile form."""
    Fn = _fn()
    torch.manual_seed(6)
    w = torch.randn(O, I, K, device="cuda")
    wp = torch.empty(O, K, I, device="cuda")
    Fn._lib.call("b2p_conv_weight_permute", w.data_ptr(), wp.data_ptr(), O, I, K, 0, Fn._st())
    assert torch.equal(wp, w.permute(0, 2, 1))
    back = torch.empty_like(w)
    Fn._lib.call("b2p_conv_weight_permute", wp.data_ptr(), back.data_ptr(), O, I, K, 1, Fn._st())
    assert torch.equal(back, w)


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_grouped_conv_view(mode):
    """positional conv: Conv1d(D, D, K, padding=K//2, groups=G) minus last frame as a grouped implicit GEMM."""
    Fn = _fn()
    torch.manual_seed(5)
    B, T, D, G, K = 2, 33, 32, 4, 8
    Og = Ig = D // G
    x = torch.randn(B, T, D, device="cuda")
    w = torch.randn(D, Ig, K, device="cuda") / 8
    wp = torch.empty(D, K * Ig, device="cuda")
    Fn._lib.call("b2p_conv_weight_permute", w.data_ptr(), wp.data_ptr(), D, Ig, K, 0, Fn._st())
    ref = F.conv1d(x.transpose(1, 2), w, padding=K // 2, groups=G)[:, :, :-1].transpose(1, 2)
    with Fn.precision(mode):
        out = torch.empty(B, T, D, device="cuda")
        A = Fn.conv_op(x, 0, D, T, T, 1, K // 2, Ig, T * D, True, bs1=Ig)
        Fn.gemm(B * T, Og, K * Ig, A, Fn.op(wp, 0, K * Ig, True, bs1=Og * K * Ig), out, D, cbs1=Og, nz1=G)
        _close(out, ref, mode)


# ------------------------------------------------------------------ bf16 operands (gemm16.hip)
def _b16(t):
    return t.to(torch.bfloat16).contiguous()


def _close16(out, ref, tol=5e-5):
    scale = ref.abs().max().item() + 1e-6
    err = (out.float() - ref).abs().max().item()
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (130, 72, 40), (1, 8, 8), (300, 264, 96), (257, 136, 2056),
                                   (96, 64, 8192)])
def test_bf16_operands_layouts(M, N, K):
    """LDS-DMA kernel: NT / NN / TN on bf16 operands vs fp64 products of the same bf16 values
    (exact products, fp32 accumulation); tails in M, N and K, split-K for the long-K case."""
    Fn = _fn()
    torch.manual_seed(10)
    Mp, Np = (M + 7) // 8 * 8, (N + 7) // 8 * 8
    a = _b16(torch.randn(M, K, device="cuda"))
    w = _b16(torch.randn(N, K, device="cuda"))
    b = _b16(torch.randn(K, Np, device="cuda"))
    at = _b16(torch.randn(K, Mp, device="cuda"))
    with Fn.precision("bf16"):
        out = torch.full((M, Np), float("nan"), device="cuda")
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), out, Np)
        _close16(out[:, :N], (a.double() @ w.double().t()).float())
        out2 = torch.full((M, Np), float("nan"), device="cuda")
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(b, 0, Np, False), out2, Np)
        _close16(out2[:, :N], (a.double() @ b[:, :N].double()).float())
        out3 = torch.full((M, Np), float("nan"), device="cuda")
        Fn.gemm(M, N, K, Fn.op(at, 0, Mp, False), Fn.op(b, 0, Np, False), out3, Np)
        _close16(out3[:, :N], (at[:, :M].double().t() @ b[:, :N].double()).float())


def test_bf16_epilogue_c16_and_batching():
    """Epilogue on the bf16 kernel (bias, GELU, pre_out, residual), bf16 copy output with and
    without the fp32 output, batched strides and the gathered (day) B operand + bias."""
    Fn = _fn()
    torch.manual_seed(11)
    M, N, K = 200, 96, 72
    x = _b16(torch.randn(M, K, device="cuda"))
    w = _b16(torch.randn(N, K, device="cuda") / 8)
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    ref_pre = (x.double() @ w.double().t()).float() + bias
    with Fn.precision("bf16"):
        out = torch.empty(M, N, device="cuda")
        pre = torch.empty(M, N, device="cuda")
        c16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Fn.gemm(M, N, K, Fn.op(x, 0, K, True), Fn.op(w, 0, K, True), out, N, bias=bias, act=Fn.ACT["gelu"],
                pre_out=pre, residual=res, C16=c16)
        _close16(pre, ref_pre)
        ref = F.gelu(ref_pre) + res
        _close16(out, ref, tol=1e-4)
        assert torch.equal(c16, out.to(torch.bfloat16))
        only16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Fn.gemm(M, N, K, Fn.op(x, 0, K, True), Fn.op(w, 0, K, True), None, N, bias=bias, C16=only16)
        torch.testing.assert_close(only16.float(), ref_pre, rtol=1e-2, atol=1e-2 * ref_pre.abs().max().item())
    # gathered per-sample B (inner n) + gathered bias: the day layer
    B, L, C, nd = 4, 40, 32, 6
    xs = _b16(torch.randn(B, L, C, device="cuda"))
    W = _b16(torch.randn(nd, C, C, device="cuda"))
    bb = torch.randn(nd, 1, C, device="cuda")
    day = torch.tensor([5, 0, 5, 2], device="cuda")
    o = torch.empty(B, L, C, device="cuda")
    with Fn.precision("bf16"):
        Fn.gemm(L, C, C, Fn.op(xs, 0, C, True, bs1=L * C), Fn.op(W, 0, C, False, bs1=C * C, gather=day), o, C,
                cbs1=L * C, nz1=B, bias=bb, biasbs1=C, bias_gather=day)
    ref = torch.einsum("btd,bdk->btk", xs.double(), W[day].double()).float() + bb[day]
    _close16(o, ref)


def test_bf16_implicit_unfold_view():
    """Implicit unfold (conv view on A) over a bf16 source: the GRU layer-0 projection."""
    Fn = _fn()
    from oracle.b2p2t_oracle import unfold
    torch.manual_seed(12)
    B, L, C, k, s, N = 3, 72, 16, 8, 4, 40
    T = (L - k) // s + 1
    x = _b16(torch.randn(B, L, C, device="cuda"))
    w = torch.randn(N, C * k, device="cuda")
    u = unfold(x.float().cpu(), k, s).cuda()
    wp = torch.empty(N, k * C, device="cuda")
    Fn._lib.call("b2p_conv_weight_permute", w.data_ptr(), wp.data_ptr(), N, C, k, 0, Fn._st())
    wp16 = _b16(wp)
    with Fn.precision("bf16"):
        out = torch.empty(B * T, N, device="cuda")
        Fn.gemm(B * T, N, k * C, Fn.conv_op(x, 0, C, T, L, s, 0, C, L * C, True), Fn.op(wp16, 0, k * C, True), out, N)
    _close16(out, (u.view(B * T, -1).double() @ w.to(torch.bfloat16).double().t()).float())


@pytest.mark.parametrize("M,N,K", [(300, 264, 96), (7968 // 8, 3072 // 4, 768 // 4), (1, 8, 8)])
def test_bf16_epilogue_pre16_aux16_colsum(M, N, K):
    """bf16-operand kernel epilogue extensions: bf16 pre-activation store (pre16), act' operand in
    bf16 (aux16) and the fused per-tile column sums (colsum_part -> b2p_colsum_parts) used for the
    FFN bias gradient, vs torch fp32 on the same bf16-rounded operands."""
    Fn = _fn()
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    ref_pre = a.float() @ w.float().t() + bias
    pre16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), None, N, bias=bias, pre16=pre16,
            act=Fn.ACT["gelu"], C16=out16)
    _close(pre16.float(), ref_pre, "bf16")
    _close(out16.float(), F.gelu(ref_pre), "bf16")
    # backward-style: C16 = (a w^T) * gelu'(aux16), colsum of the fp32 values
    g = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    parts = Fn.colsum_parts_buf(M, N, "cuda")
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), None, N, act_bwd=Fn.ACT["gelu"], aux16=pre16,
            C16=g, colsum_part=parts)
    x = pre16.float().requires_grad_(True)
    gl = torch.autograd.grad(F.gelu(x).sum(), x)[0]
    ref = (a.float() @ w.float().t()) * gl
    _close(g.float(), ref, "bf16")
    cs = Fn.colsum_from_parts(parts, torch.empty(N, device="cuda"))
    ref_cs = ref.sum(0)
    assert float((cs - ref_cs).abs().max()) <= 1e-3 * float(ref.abs().sum(0).max()) + 1e-4


_TILE_ENV = {"small": {"B2P_GEMM16_PP": "0", "B2P_GEMM16_K64": "0"},
             "small64": {"B2P_GEMM16_PP": "0", "B2P_GEMM16_K64": "1"},
             "big": {"B2P_GEMM16_PP": "0", "B2P_GEMM16_BIG": "1"},
             "pp": {"B2P_GEMM16_PP": "2", "B2P_GEMM16_PP192": "0"},
             "pp192": {"B2P_GEMM16_PP": "2", "B2P_GEMM16_PP192": "2"}}
_TILE_CASES = [(lay, M, N, K) for lay in ("AB", "Ab", "ab") for (M, N, K) in ((4096, 1536, 512), (3000, 1544, 776))]


@pytest.mark.parametrize("tile", ["small", "small64", "big", "pp", "pp192"])
def test_bf16_tile_configs(tile):
    """Every bf16 tile configuration (128x128x32 3-stage and 128x128x64 2-stage 4-wave; 256x128x64
    8-wave; 256x256x64 and 192x256x64 8-wave ping-pong), forced by environment (read once per process -> one subprocess per configuration),
    against torch fp32 on the same bf16 operands with a full epilogue (bias, GELU, residual, bf16
    copy, fused column sums), plus split-K and batched launches. The 192-row ping-pong tile takes
    k-contiguous A launches without column sums, so it also runs every case without them and on fp16
    operands. (mn-contiguous operands need ld % 8 == 0, so M, N are multiples of 8.)"""
    import os
    import subprocess
    import sys
    env = dict(os.environ, **_TILE_ENV[tile])
    code = ("import tests.test_gemm_gpu as t\n"
            "for c in t._TILE_CASES: t._check_tile_case(*c)\n"
            "t._check_tile_splitk_batched()\n"
            "for c in t._TILE_CASES: t._check_tile_case(*c, cs=False)\n"
            "for c in t._TILE_CASES: t._check_tile_case(*c, cs=False, f16=True)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]


def _check_tile_splitk_batched():
    Fn = _fn()
    torch.manual_seed(6)
    bf = torch.bfloat16
    # plain wide-K GEMM (split-K path when the grid is small) with beta accumulation
    M, N, K = 768, 1024, 4160
    a, w = torch.randn(K, M, device="cuda").to(bf), torch.randn(K, N, device="cuda").to(bf)
    c0 = torch.randn(M, N, device="cuda")
    out = c0.clone()
    Fn.gemm(M, N, K, Fn.op(a, 0, M, False), Fn.op(w, 0, N, False), out, N, beta=1.0)
    _close16(out, a.double().t() @ w.double() + c0.double(), 2e-6)
    # batched (nz1 = 3) k-contiguous operands
    Z, M, N, K = 3, 520, 776, 320
    a, w = torch.randn(Z, M, K, device="cuda").to(bf), torch.randn(Z, N, K, device="cuda").to(bf)
    out = torch.empty(Z, M, N, device="cuda")
    Fn.gemm(M, N, K, Fn.op(a, 0, K, True, bs1=M * K), Fn.op(w, 0, K, True, bs1=N * K), out, N, cbs1=M * N, nz1=Z)
    _close16(out, (a.double() @ w.double().transpose(1, 2)).float(), 2e-6)


def _check_tile_case(layout, M, N, K, cs=True, f16=False):
    Fn = _fn()
    torch.manual_seed(5)
    bf = torch.float16 if f16 else torch.bfloat16
    if f16 and layout != "AB":
        return
    if layout == "AB":
        a, w = torch.randn(M, K, device="cuda").to(bf), torch.randn(N, K, device="cuda").to(bf)
        A, Bo, ref = Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), a.float() @ w.float().t()
    elif layout == "Ab":
        a, w = torch.randn(M, K, device="cuda").to(bf), torch.randn(K, N, device="cuda").to(bf)
        A, Bo, ref = Fn.op(a, 0, K, True), Fn.op(w, 0, N, False), a.float() @ w.float()
    else:
        a, w = torch.randn(K, M, device="cuda").to(bf), torch.randn(K, N, device="cuda").to(bf)
        A, Bo, ref = Fn.op(a, 0, M, False), Fn.op(w, 0, N, False), a.float().t() @ w.float()
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    o16 = torch.empty(M, N, device="cuda", dtype=bf)
    parts = Fn.colsum_parts_buf(M, N, "cuda") if cs else None
    ob = None
    if f16:   # fp16 output copy plus the second (bf16) copy C16b
        o16 = torch.empty(M, N, device="cuda", dtype=torch.float16)
        ob = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Fn.gemm(M, N, K, A, Bo, out, N, bias=bias, act=Fn.ACT["gelu"], residual=res, C16=o16, c16_fp16=True, C16b=ob)
    else:
        Fn.gemm(M, N, K, A, Bo, out, N, bias=bias, act=Fn.ACT["gelu"], residual=res, C16=o16, colsum_part=parts)
    want = F.gelu(ref + bias) + res
    _close(out, want, "bf16", scale=want.abs().max().item())
    _close(o16.float(), want, "bf16", scale=want.abs().max().item())
    if ob is not None:
        assert torch.equal(ob, out.to(torch.bfloat16))
    if cs:
        csum = Fn.colsum_from_parts(parts, torch.empty(N, device="cuda"))
        assert float((csum - want.sum(0)).abs().max()) <= 1e-4 * float(want.abs().sum(0).max())


@pytest.mark.parametrize("fwd16", [False, True])
@pytest.mark.parametrize("M,N,K", [(512, 1024, 2048), (7968, 1024, 1024), (1000, 600, 4100)])
def test_auto16_staged_operands(fwd16, M, N, K):
    """fp32-operand GEMMs above the auto-16 threshold run on staged 16-bit operand copies
    (b2p_cast16_2d + the LDS-DMA kernel, fp16 MFMA under forward_f16): same operand rounding as the
    fp32-operand kernel, so both agree to fp32 accumulation-order noise; and both match torch fp32
    on the rounded operands. Layouts NT, NN, TN; an epilogue (bias + GELU + residual) on NT;
    K = 4100 (not a multiple of 8) stays on the fp32-operand kernel."""
    import wav2vec2forbrain_amd.functional as Fn
    torch.manual_seed(3)
    dt = torch.float16 if fwd16 else torch.bfloat16
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * 0.05
    b = torch.randn(K, N, device="cuda") * 0.05
    at = torch.randn(K, M, device="cuda")
    bias = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    r = lambda t: t.to(dt).float()
    cases = [
        (lambda o: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), o, N, bias=bias, act=Fn.ACT["gelu"],
                           residual=res),
         F.gelu(r(a) @ r(w).t() + bias) + res),
        (lambda o: Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(b, 0, N, False), o, N), r(a) @ r(b)),
        (lambda o: Fn.gemm(M, N, K, Fn.op(at, 0, M, False), Fn.op(b, 0, N, False), o, N), r(at).t() @ r(b)),
    ]
    old = Fn._AUTO16
    try:
        with Fn.precision("bf16"), Fn.forward_f16(fwd16):
            for run, ref in cases:
                outs = []
                for auto in (True, False):
                    Fn._AUTO16 = auto
                    o = torch.empty(M, N, device="cuda")
                    run(o)
                    outs.append(o)
                torch.cuda.synchronize()
                scale = ref.abs().max().item()
                assert (outs[0] - ref).abs().max().item() <= 2e-3 * scale
                assert (outs[0] - outs[1]).abs().max().item() <= 1e-4 * scale
    finally:
        Fn._AUTO16 = old


def test_scalar_epilogue_odd_n():
    """N % 4 != 0 takes the scalar epilogue (epilogue_store): bias, act' on an fp32 aux, residual,
    C16 copy against torch; the bf16-only extensions (pre16 / aux16 / colsum_part) refuse such shapes
    with an error instead of reading past the rows (advisor round 1)."""
    Fn = _fn()
    torch.manual_seed(8)
    M, N, K = 77, 262, 96
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    bias = torch.randn(N, device="cuda")
    aux = torch.randn(M, N, device="cuda")
    res = torch.randn(M, N, device="cuda")
    c = torch.empty(M, N, device="cuda")
    c16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    with Fn.precision("fp32"):
        Fn.gemm(M, N, K, Fn.op(a, 0, K, True), Fn.op(w, 0, K, True), c, N, bias=bias, act_bwd=Fn.ACT["gelu"], aux=aux,
                residual=res, C16=c16)
    x = aux.clone().requires_grad_(True)
    gl = torch.autograd.grad(F.gelu(x).sum(), x)[0]
    ref = (a @ w.t() + bias) * gl + res
    _close(c, ref, "fp32")
    assert torch.equal(c16, c.to(torch.bfloat16))
    a16, w16 = a.to(torch.bfloat16), w.to(torch.bfloat16)
    pre16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        Fn.gemm(M, N, K, Fn.op(a16, 0, K, True), Fn.op(w16, 0, K, True), None, N, pre16=pre16, C16=c16)


_SPLITK_CASES = [(3072, 768, 7968, "ab", 1.0, 1), (768, 768, 7968, "ab", 0.0, 1), (4096, 1024, 7968, "ab", 1.0, 1),
                 (1000, 520, 4200, "AB", 0.0, 1), (520, 776, 4160, "ab", 1.0, 2)]


def test_splitk_fixup_in_kernel_matches_reduce_launch():
    """The opt-in in-kernel split-K fix-up (B2P_SPLITK_FUSED=1, read once per process: one subprocess
    runs every case) against the reduce launch, bitwise (_check_splitk_fixup)."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, B2P_SPLITK_FUSED="1")
    code = "import tests.test_gemm_gpu as t\nfor c in t._SPLITK_CASES: t._check_splitk_fixup(*c)\n"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]


def _check_splitk_fixup(M, N, K, lay, beta, nz):
    """Split-K weight-gradient shapes: the in-kernel fix-up (the last K-slice workgroup of each tile sums
    the slabs, gemm16_impl.inc splitk_fixup) against the separate reduce launch (splitk_reduce4): the
    same slice order, so C must be bitwise equal; both against torch fp32 (beta = 1 accumulates into C,
    as the frozen weights' .grad). Ping-pong (4096 x 1024) and 128 x 128 (the rest) kernels, batched."""
    Fn = _fn()
    torch.manual_seed(9)
    bf = torch.bfloat16
    if lay == "ab":
        a = torch.randn(nz, K, M, device="cuda").to(bf)
        b = torch.randn(nz, K, N, device="cuda").to(bf)
        A, Bo = Fn.op(a, 0, M, False, bs1=K * M), Fn.op(b, 0, N, False, bs1=K * N)
        ref = a.double().transpose(1, 2) @ b.double()
    else:
        a = torch.randn(nz, M, K, device="cuda").to(bf)
        b = torch.randn(nz, N, K, device="cuda").to(bf)
        A, Bo = Fn.op(a, 0, K, True, bs1=M * K), Fn.op(b, 0, K, True, bs1=N * K)
        ref = a.double() @ b.double().transpose(1, 2)
    c0 = torch.randn(nz, M, N, device="cuda")
    outs = []
    old = Fn._SPLITK_CTR[0]
    try:
        for fused in (True, False):
            Fn._SPLITK_CTR[0] = fused
            c = c0.clone()
            Fn.gemm(M, N, K, A, Bo, c, N, cbs1=M * N, nz1=nz, beta=beta)
            outs.append(c)
        torch.cuda.synchronize()
    finally:
        Fn._SPLITK_CTR[0] = old
    assert torch.equal(outs[0], outs[1])
    want = ref + beta * c0.double()
    err = float((outs[0].double() - want).abs().max())
    assert err <= 2e-6 * float(want.abs().max()) * K ** 0.5, err
