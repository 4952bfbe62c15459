"""Per-operator parity of the HIP path (functional.*) against the CPU oracle / PyTorch fp32,
forward and backward, at sizes the oracle finishes in seconds."""
import math

import numpy as np

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _fn():
    from wav2vec2forbrain_amd import functional as Fn
    return Fn


def _rel(a, b):
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-12)


@pytest.mark.parametrize("n", [32 * 1024 * 256, 1001])
def test_act_bwd_softsign_exact(n):
    """b2p_act_bwd (the front end's softsign backward): the 16-byte form (n % 4 == 0) and the scalar form
    both equal dy * (1 / (1 + |x|)^2) in fp32, element for element."""
    Fn = _fn()
    torch.manual_seed(8)
    dy = torch.randn(n, device="cuda")
    x = torch.randn(n, device="cuda") * 3
    out = torch.empty_like(dy)
    Fn._lib.call("b2p_act_bwd", dy.data_ptr(), x.data_ptr(), out.data_ptr(), n, Fn.ACT["softsign"], Fn._st())
    d = 1.0 + x.abs()
    assert torch.equal(out, dy * (1.0 / (d * d)))


def test_layernorm_fwd_bwd():
    Fn = _fn()
    torch.manual_seed(0)
    for cols in (64, 768, 1024):
        x = torch.randn(37, cols, device="cuda") * 3 + 1
        g = torch.randn(cols, device="cuda")
        b = torch.randn(cols, device="cuda")
        y, mean, rstd = Fn._ln_fwd(x, g, b, 1e-5)
        xr = x.detach().clone().requires_grad_(True)
        gr = g.clone().requires_grad_(True)
        br = b.clone().requires_grad_(True)
        yr = F.layer_norm(xr, (cols,), gr, br, 1e-5)
        assert _rel(y, yr) < 1e-5
        dy = torch.randn_like(y)
        dx, dg, db, _ = Fn._ln_bwd(dy, x, g, mean, rstd)
        gx, gg, gb = torch.autograd.grad(yr, (xr, gr, br), dy)
        assert _rel(dx, gx) < 1e-4 and _rel(dg, gg) < 1e-4 and _rel(db, gb) < 1e-4


def test_softmax_fwd_bwd_with_dropout():
    Fn = _fn()
    torch.manual_seed(1)
    rows, n, ld = 50, 249, 252
    S = torch.randn(rows, ld, device="cuda") * 3
    P = torch.empty_like(S)
    Pd = torch.empty_like(S)
    Fn._lib.call("b2p_softmax_fwd", S.data_ptr(), P.data_ptr(), Pd.data_ptr(), rows, n, ld, 0.1, 77, Fn._st())
    ref = torch.softmax(S[:, :n], -1)
    assert _rel(P[:, :n], ref) < 1e-5
    keep = Pd[:, :n] != 0
    torch.testing.assert_close(Pd[:, :n][keep], ref[keep] / 0.9, rtol=1e-5, atol=1e-7)
    dPd = torch.randn(rows, ld, device="cuda")
    dS = torch.empty_like(S)
    Fn._lib.call("b2p_softmax_bwd", P.data_ptr(), dPd.data_ptr(), dS.data_ptr(), rows, n, ld, 0.1, 77, Fn._st())
    sr = S[:, :n].clone().requires_grad_(True)
    pr = torch.softmax(sr, -1) * keep.float() / 0.9
    (g,) = torch.autograd.grad(pr, sr, dPd[:, :n])
    assert _rel(dS[:, :n], g) < 1e-4


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ctc_vs_torch(seed):
    Fn = _fn()
    torch.manual_seed(seed)
    B, T, C, S = 5, 60, 32, 20
    logits = torch.randn(B, T, C, device="cuda") * 2
    tl = torch.randint(0, S + 1, (B,))
    tgt = torch.randint(1, C, (B, S))
    il = torch.randint(T // 2, T + 1, (B,)).to(torch.int32)
    if seed == 2:
        tl[0], il[0] = 20, 10        # infeasible -> zero_infinity
        tgt[1, :] = 5                 # repeated labels
    loss = Fn.ctc_loss(logits, tgt.cuda(), il.cuda(), tl.cuda())
    lr = logits.detach().cpu().double().requires_grad_(True)
    ref = F.ctc_loss(lr.log_softmax(-1).transpose(0, 1), tgt, il.long(), tl, blank=0, reduction="mean",
                     zero_infinity=True)
    (g,) = torch.autograd.grad(ref, lr)
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item()) + 1e-6
    lg = logits.clone().requires_grad_(True)
    Fn.ctc_loss(lg, tgt.cuda(), il.cuda(), tl.cuda()).backward()
    assert _rel(lg.grad.cpu().double(), g) < 1e-4


@pytest.mark.parametrize("unfold", [False, True])
@pytest.mark.parametrize("h0", [False, True])
@pytest.mark.parametrize("B,H", [(5, 32), (13, 512)])
def test_gru_layer(unfold, h0, B, H):
    """Per-step GRU kernels (csrc/gru.hip: fp32 mode, and the H = 512 Conformer encoder in every
    mode) vs the oracle GRU; B = 13 leaves a partial 8-row batch block."""
    Fn = _fn()
    from oracle.b2p2t_oracle import gru_direction, unfold as unfold_ref
    torch.manual_seed(3)
    if unfold:
        L, C, k, s = 60, 16, 8, 4
        xsrc = torch.randn(B, L, C)
        x_ref = unfold_ref(xsrc, k, s)
        x_in = Fn.Unfolded(xsrc.cuda(), k, s)
    else:
        T, IN = 23, 48
        xsrc = torch.randn(B, T, IN)
        x_ref = xsrc
        x_in = xsrc.cuda()
    IN = x_ref.shape[-1]
    ws = []
    for d in range(2):
        ws += [torch.randn(3 * H, IN) / math.sqrt(IN), torch.randn(3 * H, H) / math.sqrt(H), torch.randn(3 * H) * 0.1,
               torch.randn(3 * H) * 0.1]
    hz = torch.randn(2, B, H) if h0 else None
    # reference
    wr = [w.clone().requires_grad_(True) for w in ws]
    xr = xsrc.clone().requires_grad_(True)
    xin_ref = unfold_ref(xr, k, s) if unfold else xr
    hr = hz.clone().requires_grad_(True) if h0 else None
    outs = [gru_direction(xin_ref, *wr[4 * d:4 * d + 4], hr[d] if h0 else None, d == 1) for d in range(2)]
    ref = torch.cat(outs, -1)
    dout = torch.randn_like(ref)
    refg = torch.autograd.grad(ref, [xr, *wr] + ([hr] if h0 else []), dout)
    # HIP
    with Fn.precision("fp32"):
        wg = [w.cuda().requires_grad_(True) for w in ws]
        if unfold:
            xs = xsrc.cuda().requires_grad_(True)
            x_in = Fn.Unfolded(xs, k, s)
        else:
            xs = xsrc.cuda().requires_grad_(True)
            x_in = xs
        hg = hz.cuda().requires_grad_(True) if h0 else None
        out = Fn.gru_layer(x_in, H, 2, wg, hg)
        assert _rel(out.cpu(), ref) < 1e-4
        got = torch.autograd.grad(out, [xs, *wg] + ([hg] if h0 else []), dout.cuda())
    for a, b in zip(got, refg):
        assert _rel(a.cpu(), b) < 2e-4


@pytest.mark.parametrize("H,B,T,h0,unfold", [(32, 3, 17, True, False), (64, 5, 23, True, False), (128, 20, 40, False, False),
                                               (256, 33, 57, True, False), (256, 32, 249, False, True),
                                               (384, 20, 40, True, False), (512, 33, 57, True, False),
                                               (512, 32, 249, False, True), (256, 5, 57, True, "ragged"),
                                               (512, 7, 30, False, "ragged")])
@pytest.mark.parametrize("f16", [False, True])
def test_gru_layer_bf16_persistent(H, B, T, h0, unfold, f16):
    """bf16 mode: the persistent MFMA recurrences — one CU per (direction, 16 rows) for H <= 256
    (csrc/gru16.hip), H/64 CUs exchanging the state through L2 for H = 384 / 512 (csrc/grumc.hip,
    the Conformer encoder's H = 512) — vs the fp32 oracle GRU (nn.GRU semantics). 16-bit MFMA
    operands -> relative L2 tolerance 2e-2 on outputs and every gradient; B not a multiple of the
    16-row tile; both directions; optional h0. unfold: layer 0 over the implicit Unfold view (L a
    multiple of the stride: overlapping-row GEMM operands, no col2im) or, "ragged", over an L that is
    not (the materialised fallback). f16: the forward under Fn.forward_f16 (fp16 projection operands,
    as the models run their brain encoder) — the outputs then within 4e-3 (the recurrence's fp16
    operands: 3 more significant bits than bf16)."""
    Fn = _fn()
    from oracle.b2p2t_oracle import gru_direction, unfold as unfold_ref
    torch.manual_seed(11)
    if unfold:
        C, k, s = 16, 32, 4
        L = (T - 1) * s + k + (2 if unfold == "ragged" else 0)
        xsrc = torch.randn(B, L, C)
        x_ref_fn = lambda x: unfold_ref(x, k, s)
    else:
        IN = 48
        xsrc = torch.randn(B, T, IN)
        x_ref_fn = lambda x: x
    IN = x_ref_fn(xsrc).shape[-1]
    ws = []
    for d in range(2):
        ws += [torch.randn(3 * H, IN) / math.sqrt(IN), torch.randn(3 * H, H) / math.sqrt(H),
               torch.randn(3 * H) * 0.1, torch.randn(3 * H) * 0.1]
    hz = torch.randn(2, B, H) if h0 else None
    wr = [w.clone().requires_grad_(True) for w in ws]
    xr = xsrc.clone().requires_grad_(True)
    hr = hz.clone().requires_grad_(True) if h0 else None
    xin = x_ref_fn(xr)
    ref = torch.cat([gru_direction(xin, *wr[4 * d:4 * d + 4], hr[d] if h0 else None, d == 1) for d in range(2)], -1)
    dout = torch.randn_like(ref)
    refg = torch.autograd.grad(ref, [xr, *wr] + ([hr] if h0 else []), dout)
    with Fn.precision("bf16"):
        wg = [w.cuda().requires_grad_(True) for w in ws]
        xs = xsrc.cuda().requires_grad_(True)
        x_in = Fn.Unfolded(xs, k, s) if unfold else xs
        hg = hz.cuda().requires_grad_(True) if h0 else None
        with Fn.forward_f16(f16):
            out = Fn.gru_layer(x_in, H, 2, wg, hg)
        assert _rel(out.detach().cpu(), ref.detach()) < (4e-3 if f16 else 2e-2)
        got = torch.autograd.grad(out, [xs, *wg] + ([hg] if h0 else []), dout.cuda())
    for i, (a, b) in enumerate(zip(got, refg)):
        assert _rel(a.cpu(), b) < 3e-2, i


def _mix32(x):
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7feb352d)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846ca68b)
    return x ^ (x >> np.uint32(16))


def _keep_mask_ref(seed, p, B, nh, T):
    """numpy restatement of the dropout keep mask (csrc/common.h b2p_keep over the attention element
    index ((b*nh + h)*T + q)*TP + key, TP = T rounded up to even): (B, nh, T, T) bool."""
    with np.errstate(over="ignore"):
        k = np.uint32(seed & 0xFFFFFFFF) ^ _mix32(np.uint32(((seed >> 32) + 0x9E3779B9) & 0xFFFFFFFF))
        TP = T + (T & 1)
        row = np.arange(B * nh * T, dtype=np.uint64)[:, None] * np.uint64(TP)
        idx = (row + np.arange(T, dtype=np.uint64)[None, :]).astype(np.uint32)
        h = _mix32(_mix32((idx >> np.uint32(1)) ^ k) + k)
        half = np.where(idx & np.uint32(1), h >> np.uint32(16), h & np.uint32(0xFFFF))
    thr = int(float(np.float32(p)) * 4294967296.0)   # b2p_dropout_threshold of the float32 p
    thr16 = (thr >> 16) + ((thr >> 15) & 1)
    return (half >= thr16).reshape(B, nh, T, T)


@pytest.mark.parametrize("B,T,nh,p", [(2, 249, 12, 0.0), (2, 249, 12, 0.1), (3, 100, 4, 0.1), (1, 17, 2, 0.0),
                                       (2, 256, 3, 0.1), (2, 313, 4, 0.1), (1, 257, 2, 0.0), (1, 512, 2, 0.1),
                                       (1, 241, 2, 0.1), (1, 240, 2, 0.1)])
@pytest.mark.parametrize("variant", ["hash", "mask", "epoch", "f16"])
def test_fused_attention_bf16_vs_fp32_core(B, T, nh, p, variant):
    """csrc/attn16.hip (bf16 MFMA, scores on-chip) vs the unfused fp32 attention core (GEMM ->
    softmax/dropout kernel -> GEMM) on the same bf16-rounded q/k/v and the SAME dropout mask
    (both hash ((b*nh+h)*T+q)*T+key). Tolerance: relative L2 1e-2 on O, 2e-2 on dQ/dK/dV.
    variant: hash = backward re-hashes the mask; mask = backward reads the forward's keep bits
    (must equal the re-hashed result bit for bit); epoch = both paths under a graph-replay seed
    counter (the fused forward, fused backward and unfused kernels must offset the seed alike);
    f16 = the bf16 precision mode's default: fp16 forward operands (b2p_attn16_fwd_f16, O in fp16 plus
    its bf16 copy) and the backward recomputing the scores from them (b2p_attn16_bwd_f16).
    T' in 257..512 runs the 512-key kernels (K / V 128 KB of LDS; no stored keep mask, the backward
    rehashes; dQ recomputes the scores in a second pass), T' = 313 being a 1,280-bin window."""
    import ctypes
    Fn = _fn()
    torch.manual_seed(7)
    dh = 64
    D = nh * dh
    qkv = (torch.randn(B * T, 3 * D) * 0.7).to(torch.bfloat16).float().cuda()
    dO = torch.randn(B * T, D).to(torch.bfloat16).float().cuda()
    seed = 1234
    ctr = torch.full((1,), 7, dtype=torch.int64, device="cuda")
    lib = Fn._lib.load()
    if variant == "epoch":
        Fn._lib.check(lib.b2p_set_seed_epoch(ctypes.c_void_p(ctr.data_ptr())), "set_seed_epoch")
    try:
        with Fn.precision("fp32"):
            P, Pd, O = Fn._attn_core_fwd(qkv, B, T, nh, dh, p, seed)
            dref = Fn._attn_core_bwd(qkv, P, Pd, dO, B, T, nh, dh, p, seed)
        if variant == "f16":
            q16 = qkv.to(torch.float16)
            Oh, O16, lse2, mask = Fn._attn16_fwd_f16(q16, B, T, nh, dh, p, seed)
            assert float((Oh.float() - O16.float()).norm()) <= 1e-2 * float(Oh.float().norm())
        else:
            q16 = qkv.to(torch.bfloat16)
            O16, lse2, mask = Fn._attn16_fwd(q16, B, T, nh, dh, p, seed, want_mask=True)
        dq32, dq16 = Fn._attn16_bwd(q16, dO.to(torch.bfloat16), lse2, B, T, nh, dh, p, seed,
                                    mask=mask if variant in ("mask", "f16") else None)
        if variant == "mask" and p > 0 and mask is not None:
            h32, _ = Fn._attn16_bwd(q16, dO.to(torch.bfloat16), lse2, B, T, nh, dh, p, seed)
            # the keep bits the forward stored are the hash mask, bit for bit (integer check against
            # a numpy restatement of b2p_keep); the two backward forms then differ only by the
            # compiler's fp contraction of the identical arithmetic
            words = mask.cpu().numpy().view(np.uint32)          # (B, nh, T, 8): 32 bytes per query row
            keys = np.arange(256)
            w = (keys >> 7) + 2 * ((keys >> 2) & 3)             # byte 8*g + c, g = (key>>2)&3, c = key>>5
            sh = (8 * ((keys >> 5) & 3) + 4 * ((keys >> 4) & 1) + (keys & 3)).astype(np.uint32)
            bits = ((words[..., w] >> sh) & 1)[..., :T]
            np.testing.assert_array_equal(bits, _keep_mask_ref(seed, p, B, nh, T).astype(np.uint32))
            assert float((h32 - dq32).norm()) <= 1e-5 * float(dq32.norm())
        torch.cuda.synchronize()
    finally:
        Fn._lib.check(lib.b2p_set_seed_epoch(None), "set_seed_epoch")
    rel = lambda a, b: float((a.float() - b).norm() / b.norm())
    assert rel(O16, O) < 1e-2
    for i, name in enumerate(("dQ", "dK", "dV")):
        sl = slice(i * D, (i + 1) * D)
        assert rel(dq32[:, sl], dref[:, sl]) < 2e-2, name
        assert rel(dq16[:, sl], dref[:, sl]) < 2e-2, name
    # lse2 = log2 sum exp(scale*s) per row
    s = torch.einsum("bhqd,bhkd->bhqk", qkv[:, :D].view(B, T, nh, dh).permute(0, 2, 1, 3),
                     qkv[:, D:2 * D].view(B, T, nh, dh).permute(0, 2, 1, 3)) * dh ** -0.5
    ref_lse2 = torch.logsumexp(s, -1) / math.log(2.0)
    assert float((lse2 - ref_lse2).abs().max()) < 2e-2


@pytest.mark.parametrize("B,T,nh", [(2, 249, 12), (1, 17, 2), (2, 256, 3), (1, 241, 2), (3, 240, 2), (1, 1, 1)])
@pytest.mark.parametrize("half", [True, False])
@pytest.mark.parametrize("epoch", [False, True])
def test_attention_keep_masks_drawn_ahead(B, T, nh, half, epoch):
    """b2p_attn16_keep_masks (the encoder's masks drawn ahead beside the GRU, functional.attn_keep_plan)
    against the masks the storing forwards draw: layer l's block equals, word for word, the mask
    b2p_attn16_fwd[_f16] stores with seed l (with and without the graph-replay step counter), and the
    forward that reads it (b2p_attn16_fwd[_f16]_keep) writes O, its bf16 copy and lse2 bitwise equal to
    the storing forward's."""
    import ctypes
    Fn = _fn()
    lib = Fn._lib.load()
    torch.manual_seed(5)
    dh, p = 64, 0.1
    D = nh * dh
    qkv = (torch.randn(B * T, 3 * D) * 0.7).cuda().to(torch.float16 if half else torch.bfloat16)
    seeds = [11, 2 ** 61 + 3, 977]
    ctr = torch.full((1,), 5, dtype=torch.int64, device="cuda")
    masks = torch.empty(len(seeds), B, nh, T, 8, device="cuda", dtype=torch.int32)
    arr = (ctypes.c_uint64 * len(seeds))(*seeds)
    if epoch:
        Fn._lib.check(lib.b2p_set_seed_epoch(ctypes.c_void_p(ctr.data_ptr())), "set_seed_epoch")
    try:
        Fn._lib.call("b2p_attn16_keep_masks", masks.data_ptr(), ctypes.addressof(arr), len(seeds), B, T, nh, p,
                     Fn._st())
        for l, seed in enumerate(seeds):
            if half:
                Oh, Ob, lse2, mask = Fn._attn16_fwd_f16(qkv, B, T, nh, dh, p, seed)
                Oh2, Ob2, lse22 = torch.empty_like(Oh), torch.empty_like(Ob), torch.empty_like(lse2)
                Fn._lib.call("b2p_attn16_fwd_f16_keep", qkv.data_ptr(), Oh2.data_ptr(), Ob2.data_ptr(),
                             lse22.data_ptr(), B, T, nh, dh, float(dh ** -0.5), p, masks[l].data_ptr(), Fn._st())
                assert torch.equal(Oh, Oh2) and torch.equal(Ob, Ob2) and torch.equal(lse2, lse22)
            else:
                O16, lse2, mask = Fn._attn16_fwd(qkv, B, T, nh, dh, p, seed, want_mask=True)
                O2, lse22 = torch.empty_like(O16), torch.empty_like(lse2)
                Fn._lib.call("b2p_attn16_fwd_keep", qkv.data_ptr(), O2.data_ptr(), lse22.data_ptr(), B, T, nh, dh,
                             float(dh ** -0.5), p, masks[l].data_ptr(), Fn._st())
                assert torch.equal(O16, O2) and torch.equal(lse2, lse22)
            assert torch.equal(mask, masks[l]), l
        torch.cuda.synchronize()
    finally:
        Fn._lib.check(lib.b2p_set_seed_epoch(None), "set_seed_epoch")


@pytest.mark.parametrize("B,T,nh,p", [(2, 249, 12, 0.1), (3, 100, 4, 0.0), (1, 17, 2, 0.1), (2, 256, 3, 0.1),
                                       (1, 241, 2, 0.1), (2, 313, 4, 0.1), (1, 512, 2, 0.0)])
@pytest.mark.parametrize("form", ["f16_mask", "bf16_hash"])
def test_attention_dkv_paired_tiles_bitwise(B, T, nh, p, form):
    """The paired-key-tile dK/dV kernel (attn16_bwd_dkv2_k, the default) against the per-tile kernel
    (b2p_attn16_dkv_variant(0)): same accumulation order per key tile, so dQ/dK/dV are bitwise equal
    (fp32 and bf16 outputs), at T' with partial tiles, a wave whose second tile lies beyond T', and the
    512-key kernels."""
    Fn = _fn()
    lib = Fn._lib.load()
    torch.manual_seed(11)
    dh = 64
    D = nh * dh
    qkv = (torch.randn(B * T, 3 * D) * 0.7).cuda()
    dO = torch.randn(B * T, D).to(torch.bfloat16).cuda()
    seed = 99
    if form == "f16_mask":
        q16 = qkv.to(torch.float16)
        _, _, lse2, mask = Fn._attn16_fwd_f16(q16, B, T, nh, dh, p, seed)
    else:
        q16 = qkv.to(torch.bfloat16)
        _, lse2 = Fn._attn16_fwd(q16, B, T, nh, dh, p, seed)
        mask = None
    outs = []
    try:
        for v in (1, 0):
            Fn._lib.check(lib.b2p_attn16_dkv_variant(v), "dkv_variant")
            outs.append(Fn._attn16_bwd(q16, dO, lse2, B, T, nh, dh, p, seed, mask=mask))
        torch.cuda.synchronize()
    finally:
        Fn._lib.check(lib.b2p_attn16_dkv_variant(1), "dkv_variant")
    (a32, a16), (b32, b16) = outs
    assert torch.equal(a32, b32) and torch.equal(a16, b16)
    assert float(a32[:, D:].abs().sum()) > 0


def test_front_end():
    Fn = _fn()
    from oracle.b2p2t_oracle import gaussian_taps, gaussian_smooth, day_linear_softsign
    torch.manual_seed(4)
    B, L, C = 3, 64, 256
    x = torch.randn(B, L, C)
    day = torch.tensor([3, 17, 3])
    W = torch.eye(C).expand(24, C, C).clone() + 0.05 * torch.randn(24, C, C)
    bias = 0.1 * torch.randn(24, 1, C)
    for sigma in (0.3, 1.529):
        taps = gaussian_taps(sigma)
        Wr, br = W.clone().requires_grad_(True), bias.clone().requires_grad_(True)
        ref = day_linear_softsign(gaussian_smooth(x, taps), day, Wr, br)
        ds = torch.randn_like(ref)
        gW, gb = torch.autograd.grad(ref, (Wr, br), ds)
        with Fn.precision("fp32"):
            Wg, bg = W.cuda().requires_grad_(True), bias.cuda().requires_grad_(True)
            out = Fn.front_end(x.cuda(), day.cuda(), Wg, bg, taps.cuda())
            assert _rel(out.cpu(), ref) < 1e-5
            hW, hb = torch.autograd.grad(out, (Wg, bg), ds.cuda())
        assert _rel(hW.cpu(), gW) < 1e-4 and _rel(hb.cpu(), gb) < 1e-4


def test_pos_conv_ln():
    Fn = _fn()
    from oracle.b2p2t_oracle import pos_conv, layer_norm, OracleConfig
    torch.manual_seed(5)
    B, T, D, G, K = 2, 41, 64, 4, 16
    cfg = OracleConfig(num_conv_pos_embeddings=K, num_conv_pos_embedding_groups=G)
    e = torch.randn(B, T, D)
    g = 1 + 0.1 * torch.randn(1, 1, K)
    v = torch.randn(D, D // G, K)
    cb = 0.05 * torch.randn(D)
    lg, lb = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    ts = [t.clone().requires_grad_(True) for t in (e, g, v, cb, lg, lb)]
    sd = {"p.conv.parametrizations.weight.original0": ts[1], "p.conv.parametrizations.weight.original1": ts[2],
          "p.conv.bias": ts[3]}
    ref = layer_norm(ts[0] + pos_conv(ts[0], sd, "p.", cfg), ts[4], ts[5], 1e-5)
    dy = torch.randn_like(ref)
    refg = torch.autograd.grad(ref, ts, dy)
    with Fn.precision("fp32"):
        tg = [t.cuda().requires_grad_(True) for t in (e, g, v, cb, lg, lb)]
        out = Fn.pos_conv_ln(*tg, G, 1e-5, 0.0, False)
        assert _rel(out.cpu(), ref) < 1e-4
        got = torch.autograd.grad(out, tg, dy.cuda())
    for i, (a, b) in enumerate(zip(got, refg)):
        assert _rel(a.cpu(), b) < 5e-4, i


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_encoder_layer(mode):
    Fn = _fn()
    from oracle.b2p2t_oracle import encoder_layer, OracleConfig
    torch.manual_seed(6)
    B, T, D, nh, Ff = 2, 45, 64, 4, 128
    cfg = OracleConfig(hidden_size=D, num_attention_heads=nh, intermediate_size=Ff)
    names = ["attention.q_proj.weight", "attention.q_proj.bias", "attention.k_proj.weight", "attention.k_proj.bias",
             "attention.v_proj.weight", "attention.v_proj.bias", "attention.out_proj.weight", "attention.out_proj.bias",
             "layer_norm.weight", "layer_norm.bias", "feed_forward.intermediate_dense.weight",
             "feed_forward.intermediate_dense.bias", "feed_forward.output_dense.weight",
             "feed_forward.output_dense.bias", "final_layer_norm.weight", "final_layer_norm.bias"]
    shapes = [(D, D), (D,), (D, D), (D,), (D, D), (D,), (D, D), (D,), (D,), (D,), (Ff, D), (Ff,), (D, Ff), (D,), (D,), (D,)]
    vals = []
    for n, s in zip(names, shapes):
        r = torch.randn(*s)
        vals.append(1 + 0.1 * r if "norm.weight" in n else (0.05 * r if len(s) == 1 else r / math.sqrt(s[1])))
    x = torch.randn(B, T, D)
    pr = [v.clone().requires_grad_(True) for v in vals]
    xr = x.clone().requires_grad_(True)
    ref = encoder_layer(xr, {"l." + n: p for n, p in zip(names, pr)}, "l.", cfg, False)
    dy = torch.randn_like(ref)
    refg = torch.autograd.grad(ref, [xr] + pr, dy)
    tol = 2e-4 if mode == "fp32" else 3e-2
    with Fn.precision(mode):
        pg = [v.cuda().requires_grad_(True) for v in vals]
        xg = x.cuda().requires_grad_(True)
        out = Fn.encoder_layer(xg, pg, nh, 1e-5, 0.0, 0.0, 0.0, False)
        assert _rel(out.cpu(), ref) < tol
        got = torch.autograd.grad(out, [xg] + pg, dy.cuda())
    for i, (a, b) in enumerate(zip(got, refg)):
        if i == 4:   # k_proj bias: gradient is mathematically zero (softmax shift invariance)
            assert a.abs().max().item() < tol * refg[0].abs().max().item() + 1e-6
            continue
        assert _rel(a.cpu(), b) < tol * 5, (i, _rel(a.cpu(), b))


def test_encoder_layer_dropout_train_mode():
    """train-mode: outputs finite, dropout active, backward consistent with forward masks
    (finite-difference check of the directional derivative)."""
    Fn = _fn()
    torch.manual_seed(7)
    B, T, D, nh, Ff = 2, 20, 32, 2, 64
    shapes = [(D, D), (D,), (D, D), (D,), (D, D), (D,), (D, D), (D,), (D,), (D,), (Ff, D), (Ff,), (D, Ff), (D,), (D,), (D,)]
    ps = [(torch.randn(*s) / math.sqrt(s[-1])).cuda().double().float() for s in shapes]
    ps[8] = torch.ones(D, device="cuda"); ps[14] = torch.ones(D, device="cuda")
    x = torch.randn(B, T, D, device="cuda")
    cfg_seeds = (11, 12, 13, 14)
    cfg = (nh, 1e-5, 0.1, 0.1, 0.1, cfg_seeds)
    with Fn.precision("fp32"):
        xg = x.clone().requires_grad_(True)
        out = Fn._EncoderLayer.apply(xg, cfg, *ps)
        dy = torch.randn_like(out)
        (gx,) = torch.autograd.grad(out, xg, dy)
        d = torch.randn_like(x)
        eps = 1e-2
        fp = Fn._EncoderLayer.apply(x + eps * d, cfg, *ps)
        fm = Fn._EncoderLayer.apply(x - eps * d, cfg, *ps)
        fd = ((fp - fm) * dy).sum() / (2 * eps)
        an = (gx * d).sum()
    assert torch.isfinite(out).all()
    assert abs(fd.item() - an.item()) <= 2e-2 * abs(an.item()) + 1e-3


def test_adam_matches_torch():
    from wav2vec2forbrain_amd.optim import HipAdam
    torch.manual_seed(8)
    shapes = [(300, 70), (5,), (24, 1, 256)]
    ps1 = [torch.nn.Parameter(torch.randn(*s, device="cuda")) for s in shapes]
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps1]
    o1 = torch.optim.Adam(ps1, lr=1e-3, weight_decay=0.01, eps=1e-8)
    o2 = HipAdam(ps2, lr=1e-3, weight_decay=0.01, eps=1e-8)
    for step in range(5):
        gs = [torch.randn_like(p) for p in ps1]
        for p, g in zip(ps1, gs):
            p.grad = g.clone()
        for p, g in zip(ps2, gs):
            p.grad = g.clone()
        o1.step()
        o2.step()
    for a, b in zip(ps1, ps2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_accum_recs_multi_tensor():
    """b2p_accum_recs (one launch, records by value) == per-tensor dst += src, incl. > 96 records
    (two launches), an empty tensor and one larger than the grid stride; and the deferred small-grad
    path of functional.flush_wgrad (p.grad None -> takes g; else accumulated) equals torch's adds."""
    import ctypes
    Fn = _fn()
    torch.manual_seed(11)
    sizes = [768, 1, 3072, 0, 5000000] + [int(n) for n in torch.randint(1, 3000, (110,))]
    dst = [torch.randn(n, device="cuda") for n in sizes]
    src = [torch.randn(n, device="cuda") for n in sizes]
    ref = [d + s for d, s in zip(dst, src)]
    recs = []
    for d, s in zip(dst, src):
        recs += [d.data_ptr(), s.data_ptr(), d.numel()]
    arr = (ctypes.c_int64 * len(recs))(*recs)
    Fn._lib.call("b2p_accum_recs", arr, len(sizes), Fn._st())
    torch.cuda.synchronize()
    for a, b in zip(dst, ref):
        assert torch.equal(a, b)
    # through the deferral queue
    ps = [torch.nn.Parameter(torch.randn(7, 5, device="cuda")) for _ in range(4)]
    ps[0].grad = None
    for p in ps[1:]:
        p.grad = torch.randn_like(p)
    gs = [torch.randn_like(p) for p in ps]
    want = [g.clone() if p.grad is None else p.grad + g for p, g in zip(ps, gs)]
    for p, g in zip(ps, gs):
        Fn._defer_acc(p, g)
    Fn.join_wgrad()
    torch.cuda.synchronize()
    for p, w in zip(ps, want):
        assert torch.equal(p.grad, w)


@pytest.mark.parametrize("B,T,D,K", [(2, 249, 1024, 31), (1, 65, 70, 31), (3, 130, 128, 5), (1, 3, 64, 31)])
def test_dwconv_tiled_shapes(B, T, D, K):
    """LDS-tiled depthwise conv (fwd, dx, dw) vs torch fp32 conv1d at the Conformer-large shape and
    at ragged tails: T not a multiple of the 64-frame tile, channels not a multiple of 64, T < K."""
    Fn = _fn()
    torch.manual_seed(12)
    x = torch.randn(B, T, D, device="cuda")
    w = torch.randn(D, 1, K, device="cuda")
    xc, wc = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    yc = F.conv1d(xc.transpose(1, 2), wc, padding=(K - 1) // 2, groups=D).transpose(1, 2)
    y = torch.empty(B, T, D, device="cuda")
    Fn._lib.call("b2p_dwconv_fwd", x.data_ptr(), w.data_ptr(), y.data_ptr(), B, T, D, K, Fn._st())
    gy = torch.randn_like(yc)
    gxc, gwc = torch.autograd.grad(yc, (xc, wc), gy)
    dx = torch.empty(B, T, D, device="cuda")
    dw = torch.empty(D, 1, K, device="cuda")
    ws = torch.empty(int(Fn._lib.load().b2p_dwconv_bwd_workspace(B, T, D, K)), device="cuda")
    Fn._lib.call("b2p_dwconv_bwd", x.data_ptr(), w.data_ptr(), gy.contiguous().data_ptr(), dx.data_ptr(),
                 dw.data_ptr(), B, T, D, K, ws.data_ptr(), Fn._st())
    torch.cuda.synchronize()
    assert _rel(y, yc) < 1e-5 and _rel(dx, gxc) < 1e-5 and _rel(dw, gwc) < 1e-5


def test_conformer_elementwise_kernels():
    """rotary (fwd + transpose), GLU, depthwise conv, BatchNorm+SiLU against torch fp32."""
    Fn = _fn()
    from oracle.b2p2t_oracle import rotary_apply
    torch.manual_seed(9)
    B, T, nh, dh, K = 2, 37, 4, 16, 7
    D = nh * dh
    x = torch.randn(B, T, D)
    keep = []                       # device copies must outlive the raw-pointer calls

    def dev(t):
        d = t.cuda()
        keep.append(d)
        return d.data_ptr()
    # rotary
    cos_t, sin_t = Fn.rotary_tables(T, dh, 10000, "cuda")
    out = torch.empty(B * T, D, device="cuda")
    Fn._lib.call("b2p_rotary", dev(x), cos_t.data_ptr(), sin_t.data_ptr(), out.data_ptr(), B, T, nh, dh,
                 D, 0, Fn._st())
    xr = x.clone().requires_grad_(True)
    ref = rotary_apply(xr, nh, 10000)
    assert _rel(out.view(B, T, D).cpu(), ref) < 1e-5
    g = torch.randn_like(ref)
    (gx,) = torch.autograd.grad(ref, xr, g)
    back = torch.empty(B * T, D, device="cuda")
    Fn._lib.call("b2p_rotary", dev(g), cos_t.data_ptr(), sin_t.data_ptr(), back.data_ptr(), B, T, nh, dh,
                 D, 1, Fn._st())
    assert _rel(back.view(B, T, D).cpu(), gx) < 1e-5
    # GLU
    a = torch.randn(B * T, 2 * D)
    u = torch.empty(B * T, D, device="cuda")
    Fn._lib.call("b2p_glu_fwd", dev(a), u.data_ptr(), B * T, D, Fn._st())
    ar = a.clone().requires_grad_(True)
    ur = F.glu(ar, dim=1)
    assert _rel(u.cpu(), ur) < 1e-6
    gu = torch.randn(ur.shape)
    (ga,) = torch.autograd.grad(ur, ar, gu)
    da = torch.empty(B * T, 2 * D, device="cuda")
    Fn._lib.call("b2p_glu_bwd", dev(a), dev(gu), da.data_ptr(), B * T, D, Fn._st())
    assert _rel(da.cpu(), ga) < 1e-5
    # depthwise conv
    w = torch.randn(D, 1, K)
    xc = x.clone().requires_grad_(True)
    wc = w.clone().requires_grad_(True)
    yc = F.conv1d(xc.transpose(1, 2), wc, padding=(K - 1) // 2, groups=D).transpose(1, 2)
    y = torch.empty(B, T, D, device="cuda")
    Fn._lib.call("b2p_dwconv_fwd", dev(x), dev(w), y.data_ptr(), B, T, D, K, Fn._st())
    assert _rel(y.cpu(), yc) < 1e-5
    gy = torch.randn(yc.shape)            # contiguous (B, T, D)
    gxc, gwc = torch.autograd.grad(yc, (xc, wc), gy)
    dx = torch.empty(B, T, D, device="cuda")
    dw = torch.empty(D, 1, K, device="cuda")
    ws = torch.empty(int(Fn._lib.load().b2p_dwconv_bwd_workspace(B, T, D, K)), device="cuda")
    Fn._lib.call("b2p_dwconv_bwd", dev(x), dev(w), dev(gy), dx.data_ptr(),
                 dw.data_ptr(), B, T, D, K, ws.data_ptr(), Fn._st())
    assert _rel(dx.cpu(), gxc) < 1e-5 and _rel(dw.cpu(), gwc) < 1e-5
    # BatchNorm (train) + SiLU
    M = B * T
    xb = torch.randn(M, D) * 2 + 0.5
    gam, bet = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    rm, rv = torch.zeros(D), torch.ones(D)
    xr = xb.clone().requires_grad_(True)
    gr, br = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    yr = F.silu(F.batch_norm(xr, rm_ref, rv_ref, gr, br, training=True, momentum=0.1, eps=1e-5))
    yb = torch.empty(M, D, device="cuda")
    pre = torch.empty(M, D, device="cuda")
    mean = torch.empty(D, device="cuda")
    rstd = torch.empty(D, device="cuda")
    rmg, rvg = rm.cuda(), rv.cuda()
    ws = torch.empty(int(Fn._lib.load().b2p_batchnorm_workspace(M, D)), device="cuda")
    Fn._lib.call("b2p_batchnorm_fwd", dev(xb), dev(gam), dev(bet),
                 rmg.data_ptr(), rvg.data_ptr(), yb.data_ptr(), pre.data_ptr(), mean.data_ptr(), rstd.data_ptr(), M, D,
                 1e-5, 0.1, Fn.ACT["silu"], ws.data_ptr(), Fn._st())
    assert _rel(yb.cpu(), yr) < 1e-5
    assert _rel(rmg.cpu(), rm_ref) < 1e-5 and _rel(rvg.cpu(), rv_ref) < 1e-5
    gyb = torch.randn(yr.shape)
    gx_, gg_, gb_ = torch.autograd.grad(yr, (xr, gr, br), gyb)
    dxb = torch.empty(M, D, device="cuda")
    dg = torch.empty(D, device="cuda")
    db = torch.empty(D, device="cuda")
    Fn._lib.call("b2p_batchnorm_bwd", dev(gyb), pre.data_ptr(), dev(xb), mean.data_ptr(),
                 rstd.data_ptr(), dev(gam), dxb.data_ptr(), dg.data_ptr(), db.data_ptr(), M, D,
                 Fn.ACT["silu"], ws.data_ptr(), Fn._st())
    assert _rel(dxb.cpu(), gx_) < 1e-4 and _rel(dg.cpu(), gg_) < 1e-4 and _rel(db.cpu(), gb_) < 1e-4


def test_cast_and_layernorm_bf16_copies():
    """b2p_cast_bf16 == torch RNE rounding; LayerNorm fwd/bwd bf16 copies equal the rounded fp32
    outputs they shadow."""
    Fn = _fn()
    torch.manual_seed(21)
    x = torch.randn(1003, device="cuda") * 7
    torch.testing.assert_close(Fn.cast16(x), x.to(torch.bfloat16), rtol=0, atol=0)
    rows, cols = 77, 768
    xx = torch.randn(rows, cols, device="cuda")
    g = 1 + 0.1 * torch.randn(cols, device="cuda")
    b = 0.1 * torch.randn(cols, device="cuda")
    y, y16, m, r = Fn._ln_fwd16(xx, g, b, 1e-5)
    y0, m0, r0 = Fn._ln_fwd(xx, g, b, 1e-5)
    assert torch.equal(y, y0) and torch.equal(y16, y.to(torch.bfloat16))
    dy = torch.randn(rows, cols, device="cuda")
    dx, dg, db, dxd, d16 = Fn._ln_bwd16(dy, xx, g, m, r, True, in_drop_p=0.1, in_seed=5)
    dx0, dg0, db0, dxd0 = Fn._ln_bwd(dy, xx, g, m, r, True, in_drop_p=0.1, in_seed=5)
    assert torch.equal(dx, dx0) and torch.equal(dxd, dxd0) and torch.equal(d16, dxd.to(torch.bfloat16))
    dx, dg, db, dxd, d16 = Fn._ln_bwd16(dy, xx, g, m, r, True)
    assert dxd is None and torch.equal(d16, dx.to(torch.bfloat16))


def test_encoder_layer_bf16_operands_match_fp32_path():
    """_EncoderLayer16 (bf16 operands in HBM, fused QKV) vs _EncoderLayer (fp32 operands) in
    train mode with identical dropout seeds: same masks, bf16-level agreement of output and
    every gradient; and the cached bf16 weights refresh after an in-place optimiser update."""
    Fn = _fn()
    torch.manual_seed(22)
    B, T, D, nh, Ff = 2, 37, 64, 4, 128
    shapes = [(D, D), (D,), (D, D), (D,), (D, D), (D,), (D, D), (D,), (D,), (D,), (Ff, D), (Ff,), (D, Ff), (D,), (D,), (D,)]
    ps = [(torch.randn(*s) / math.sqrt(s[-1])).cuda() for s in shapes]
    ps[8] = torch.ones(D, device="cuda"); ps[14] = torch.ones(D, device="cuda")
    x = torch.randn(B, T, D, device="cuda")
    cfg = (nh, 1e-5, 0.1, 0.1, 0.1, (31, 32, 33, 34))
    dy = torch.randn(B, T, D, device="cuda")
    res = []
    for cls, mode in ((Fn._EncoderLayer, "fp32"), (Fn._EncoderLayer16, "bf16")):
        with Fn.precision(mode):
            pg = [p.clone().requires_grad_(True) for p in ps]
            xg = x.clone().requires_grad_(True)
            out = cls.apply(xg, cfg, *pg)
            res.append([out] + list(torch.autograd.grad(out, [xg] + pg, dy)))
    for i, (a, b) in enumerate(zip(res[0], res[1])):
        if i == 5:     # k_proj bias gradient: mathematically 0 (softmax shift invariance), rounding noise
            assert b.abs().max().item() < 3e-2 * res[0][1].abs().max().item()
            continue
        assert _rel(b.cpu(), a.cpu()) < 3e-2, (i, _rel(b.cpu(), a.cpu()))
    # cache refresh: change a weight in place through a raw pointer + epoch bump
    with Fn.precision("bf16"):
        w = ps[10].clone()
        w16a = Fn.weight16(w).clone()
        Fn._lib.call("b2p_dropout", w.data_ptr(), w.data_ptr(), w.numel(), 0.5, 9, Fn._st())   # in-place write
        assert torch.equal(Fn.weight16(w), w16a)          # torch cannot see it ...
        Fn.bump_param_epoch([w])
        assert torch.equal(Fn.weight16(w), w.to(torch.bfloat16))   # ... the epoch bump can


def test_encoder_layer_f16_forward_matches_fp32_path():
    """_EncoderLayer16 under Fn.forward_f16 (fused attention, dh 64): every forward GEMM operand fp16
    (QKV / out-projection / FFN inputs and weights; the producers also write the backward's bf16
    operands) vs _EncoderLayer in fp32 with the same dropout seeds: the output within fp16 rounding
    (an order of magnitude under the bf16 forward's), every gradient at bf16 level; the layer's
    output carries both 16-bit copies for the next layer."""
    Fn = _fn()
    torch.manual_seed(23)
    B, T, D, nh, Ff = 2, 200, 128, 2, 256
    shapes = [(D, D), (D,), (D, D), (D,), (D, D), (D,), (D, D), (D,), (D,), (D,), (Ff, D), (Ff,), (D, Ff), (D,), (D,), (D,)]
    ps = [(torch.randn(*s) / math.sqrt(s[-1])).cuda() for s in shapes]
    ps[8] = torch.ones(D, device="cuda"); ps[14] = torch.ones(D, device="cuda")
    x = torch.randn(B, T, D, device="cuda")
    cfg = (nh, 1e-5, 0.1, 0.1, 0.1, (41, 42, 43, 44))
    dy = torch.randn(B, T, D, device="cuda")
    res, outs = [], []
    for cls, mode, f16 in ((Fn._EncoderLayer, "fp32", False), (Fn._EncoderLayer16, "bf16", False),
                           (Fn._EncoderLayer16, "bf16", True)):
        with Fn.precision(mode), Fn.forward_f16(f16):
            pg = [p.clone().requires_grad_(True) for p in ps]
            xg = x.clone().requires_grad_(True)
            out = cls.apply(xg, cfg, *pg)
            outs.append(out)
            res.append([out] + list(torch.autograd.grad(out, [xg] + pg, dy)))
    e16, eb = _rel(res[2][0].cpu(), res[0][0].cpu()), _rel(res[1][0].cpu(), res[0][0].cpu())
    assert e16 < 3e-3 and e16 < 0.35 * eb, (e16, eb)
    for i, (a, b) in enumerate(zip(res[0], res[2])):
        if i in (0, 5):     # output (above); k_proj bias gradient: mathematically 0
            continue
        assert _rel(b.cpu(), a.cpu()) < 3e-2, (i, _rel(b.cpu(), a.cpu()))
    o, od = outs[2], outs[2].detach()
    assert o._h16[1].dtype == torch.float16 and torch.equal(o._h16[1], od.to(torch.float16))
    assert o._b16[1].dtype == torch.bfloat16 and torch.equal(o._b16[1], od.to(torch.bfloat16))


def test_dropout_seed_epoch_counter():
    """Graph-replay seed counter (b2p_set_seed_epoch): counter 0 reproduces the eager mask, every
    b2p_seed_epoch_step gives a new mask, NULL restores eager semantics; the GEMM epilogue and the
    stand-alone dropout kernel see the same counter."""
    import ctypes
    Fn = _fn()
    lib = Fn._lib.load()
    x = torch.ones(1 << 16, device="cuda")

    def mask():
        y = torch.empty_like(x)
        Fn._lib.call("b2p_dropout", x.data_ptr(), y.data_ptr(), x.numel(), 0.5, 1234, Fn._st())
        return y != 0

    def gemm_mask():
        a = torch.ones(256, 64, device="cuda", dtype=torch.bfloat16)
        w = torch.ones(128, 64, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(256, 128, device="cuda")
        Fn.gemm(256, 128, 64, Fn.op(a, 0, 64, True), Fn.op(w, 0, 64, True), out, 128, drop_p=0.5, seed=77)
        return out != 0

    m0, g0 = mask(), gemm_mask()
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    try:
        Fn._lib.check(lib.b2p_set_seed_epoch(ctypes.c_void_p(ctr.data_ptr())), "set_seed_epoch")
        assert torch.equal(mask(), m0) and torch.equal(gemm_mask(), g0)
        Fn._lib.check(lib.b2p_seed_epoch_step(ctypes.c_void_p(ctr.data_ptr()), ctypes.c_void_p(Fn._st())), "step")
        m1, g1 = mask(), gemm_mask()
        assert int(ctr.item()) == 1
        assert not torch.equal(m1, m0) and not torch.equal(g1, g0)
        assert abs(m1.float().mean().item() - 0.5) < 0.02
    finally:
        Fn._lib.check(lib.b2p_set_seed_epoch(None), "set_seed_epoch")
    assert torch.equal(mask(), m0)


def test_pos_conv_ln_bf16_posconv16():
    """wav2vec2-base positional conv (768 channels, 16 groups of 48, 128 taps) on the bf16 slab kernels
    (csrc/posconv16.hip: forward, backward-data with the conv-bias column sums, weight gradient)
    against the CPU oracle in fp32; odd batch (a half-empty sample pair), T below the 256 cap."""
    Fn = _fn()
    from oracle.b2p2t_oracle import pos_conv, layer_norm, OracleConfig
    torch.manual_seed(15)
    B, T, D, G, K = 3, 131, 768, 16, 128
    cfg = OracleConfig(num_conv_pos_embeddings=K, num_conv_pos_embedding_groups=G, hidden_size=D)
    e = torch.randn(B, T, D)
    g = 1 + 0.1 * torch.randn(1, 1, K)
    v = torch.randn(D, D // G, K) / math.sqrt(48 * 128)
    cb = 0.05 * torch.randn(D)
    lg, lb = 1 + 0.1 * torch.randn(D), 0.1 * torch.randn(D)
    ts = [t.clone().requires_grad_(True) for t in (e, g, v, cb, lg, lb)]
    sd = {"p.conv.parametrizations.weight.original0": ts[1], "p.conv.parametrizations.weight.original1": ts[2],
          "p.conv.bias": ts[3]}
    ref = layer_norm(ts[0] + pos_conv(ts[0], sd, "p.", cfg), ts[4], ts[5], 1e-5)
    dy = torch.randn_like(ref)
    refg = torch.autograd.grad(ref, ts, dy)
    with Fn.precision("bf16"):
        assert Fn._posconv16_ok(B, T, D, D, 48, K, G)
        tg = [t.cuda().requires_grad_(True) for t in (e, g, v, cb, lg, lb)]
        out = Fn.pos_conv_ln(*tg, G, 1e-5, 0.0, False)
        got = torch.autograd.grad(out, tg, dy.cuda())

    def rl2(a, b):
        return float((a.detach().cpu() - b.detach()).norm() / b.detach().norm())
    assert rl2(out, ref) < 1e-2
    for i, (a, b) in enumerate(zip(got, refg)):
        assert rl2(a, b) < 2e-2, (i, rl2(a, b))


def test_gru_mc_direct_and_graph_replay():
    """csrc/grumc.hip through the C ABI: the multi-CU forward / backward equal the per-step fp32
    kernels (csrc/gru.hip) within bf16 operand rounding, the timeout flag stays 0, and replaying a
    captured graph of both launches (the workspace memset is a graph node, so stale tags of the
    previous replay never match) reproduces the eager results bit for bit."""
    Fn = _fn()
    from wav2vec2forbrain_amd import _lib
    torch.manual_seed(5)
    B, T, H, nd = 33, 41, 512, 2
    dev = "cuda"
    gi = torch.randn(B, T, nd * 3 * H, device=dev)
    whh = torch.randn(nd, 3 * H, H, device=dev) / math.sqrt(H)
    bhh = torch.randn(nd, 3 * H, device=dev) * 0.1
    h0 = torch.randn(nd, B, H, device=dev)
    dout = torch.randn(B, T, nd * H, device=dev)

    def run(mc):
        out = torch.empty(B, T, nd * H, device=dev)
        sv = torch.empty(B, T, nd, 4, H, device=dev)
        dgi = torch.empty(B, T, nd * 3 * H, device=dev)
        dgh = torch.empty_like(dgi)
        dh0 = torch.empty(nd, B, H, device=dev)
        if mc:
            ws = torch.empty(int(_lib.load().b2p_gru_mc_workspace(B, H, nd)), device=dev, dtype=torch.uint8)
            _lib.call("b2p_gru_fwd_mc", gi.data_ptr(), whh.data_ptr(), bhh.data_ptr(), h0.data_ptr(), out.data_ptr(),
                      sv.data_ptr(), ws.data_ptr(), B, T, H, nd, _lib.stream_ptr())
            f1 = ws[:4].clone()
            _lib.call("b2p_gru_bwd_mc", dout.data_ptr(), whh.data_ptr(), out.data_ptr(), sv.data_ptr(), h0.data_ptr(),
                      dgi.data_ptr(), dgh.data_ptr(), dh0.data_ptr(), ws.data_ptr(), B, T, H, nd, _lib.stream_ptr())
            return out, sv, dgi, dgh, dh0, torch.cat([f1, ws[:4]])
        buf = torch.empty(nd, B, H, device=dev)
        _lib.call("b2p_gru_fwd", gi.data_ptr(), whh.data_ptr(), bhh.data_ptr(), h0.data_ptr(), out.data_ptr(),
                  sv.data_ptr(), B, T, H, nd, _lib.stream_ptr())
        _lib.call("b2p_gru_bwd", dout.data_ptr(), whh.data_ptr(), out.data_ptr(), sv.data_ptr(), h0.data_ptr(),
                  dgi.data_ptr(), dgh.data_ptr(), dh0.data_ptr(), buf.data_ptr(), B, T, H, nd, _lib.stream_ptr())
        return out, sv, dgi, dgh, dh0, None

    ref = run(False)
    got = run(True)
    torch.cuda.synchronize()
    assert int(got[5].abs().sum()) == 0, "a member timed out"
    for a, r in zip(got[:5], ref[:5]):
        assert _rel(a.cpu(), r.cpu()) < 2e-2
    # graph replay: same results, every replay
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(True)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        res = run(True)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert int(res[5].abs().sum()) == 0
        for a, b in zip(res[:5], got[:5]):
            assert torch.equal(a, b)


def test_gru_mc_timeout_raises():
    """A multi-CU GRU launch whose member never publishes its state (test knob: member 1 withholds
    its exchange stores) times out instead of hanging, and the failure is not silent: the launch's
    timeout flag is folded into the persistent status word (b2p_gru_mc_status) and the next loss
    readback (functional.loss_item, the reference's per-step .item()) raises RuntimeError naming the
    recurrence. Healthy launches afterwards leave the word at 0."""
    Fn = _fn()
    from wav2vec2forbrain_amd import _lib
    torch.manual_seed(6)
    B, T, H, IN = 16, 6, 512, 64
    dev = "cuda"
    x = torch.randn(B, T, IN, device=dev, requires_grad=True)
    w = [torch.randn(3 * H, IN, device=dev) / 8, torch.randn(3 * H, H, device=dev) / math.sqrt(H),
         torch.zeros(3 * H, device=dev), torch.zeros(3 * H, device=dev)]
    Fn.check_gru_status()   # start clean
    with Fn.precision("bf16"):
        _lib.call("b2p_gru_mc_debug_withhold", 1)
        try:
            out = Fn.gru_layer(x, H, 1, w)
            loss = out.square().mean()
            torch.cuda.synchronize()
        finally:
            _lib.call("b2p_gru_mc_debug_withhold", -1)
        with pytest.raises(RuntimeError, match="multi-CU GRU recurrence timed out \\(forward of GRU layer"):
            Fn.loss_item(loss)
        assert Fn.gru_status_value() == 0   # cleared by the raise
        out = Fn.gru_layer(x, H, 1, w)
        out.square().mean().backward()
        Fn.loss_item(out.square().mean())   # healthy: no raise
    assert Fn.gru_status_value() == 0


@pytest.mark.gpu
def test_conformer_16bit_producers():
    """The Conformer's 16-bit operand producers against torch fp32: LayerNorm with its fp16/bf16 copy,
    rotary written as fp16/bf16, bf16(dropout(act(pre))) with the GEMM-epilogue mask, the fused
    output-dropout backward (bf16 copy + column sums), and the GEMM epilogue's fp16 C16 flag."""
    Fn = _fn()
    from oracle.b2p2t_oracle import rotary_apply
    torch.manual_seed(11)
    M, D, nh = 300, 256, 4
    dh = D // nh
    x = torch.randn(M, D, device="cuda")
    g, b = 1 + 0.1 * torch.randn(D, device="cuda"), 0.1 * torch.randn(D, device="cuda")
    ref = F.layer_norm(x, (D,), g, b, 1e-5)
    for half in (True, False):
        y, y16, mean, rstd, y16b = Fn._ln_fwd_x16(x, g, b, 1e-5, half, want_b16=True)
        assert y16.dtype == (torch.float16 if half else torch.bfloat16)
        assert _rel(y.cpu(), ref.cpu()) < 1e-5
        assert torch.equal(y16, y.to(y16.dtype))        # the copy is the RNE rounding of y
        assert torch.equal(y16b, y.to(torch.bfloat16))
        _, y16n, _, _ = Fn._ln_fwd_x16(x, g, b, 1e-5, half, want32=False)   # no fp32 output
        assert torch.equal(y16n, y16)
    # GLU backward written as bf16 == bf16(b2p_glu_bwd)
    a = torch.randn(M, 2 * D, device="cuda")
    du = torch.randn(M, D, device="cuda")
    da = torch.empty(M, 2 * D, device="cuda")
    Fn._lib.call("b2p_glu_bwd", a.data_ptr(), du.data_ptr(), da.data_ptr(), M, D, Fn._st())
    da16 = torch.empty(M, 2 * D, device="cuda", dtype=torch.bfloat16)
    Fn._lib.call("b2p_glu_bwd16", a.data_ptr(), du.data_ptr(), da16.data_ptr(), M, D, Fn._st())
    assert torch.equal(da16, da.to(torch.bfloat16))
    # rotary16 == b2p_rotary (fp32) rounded
    B, T = 3, 100
    h = torch.randn(B * T, D, device="cuda")
    cos_t, sin_t = Fn.rotary_tables(T, dh, 10000, "cuda")
    r32 = rotary_apply(h.view(B, T, D).cpu(), nh, 10000).view(B * T, D)
    for half in (True, False):
        r16 = Fn._rotary16(h, cos_t, sin_t, B, T, nh, dh, half)
        assert _rel(r16.float().cpu(), r32) < (1e-3 if half else 8e-3)
    # act + dropout + bf16 cast with the epilogue's mask: compare with a GEMM whose epilogue applies
    # the same act / dropout to x @ I (exact in fp32 operands)
    K = 64
    a = torch.randn(M, K, device="cuda")
    eye = torch.eye(K, device="cuda")
    pre = torch.empty(M, K, device="cuda")
    fo = torch.empty(M, K, device="cuda")
    seed = 1234
    with Fn.precision("fp32"):
        Fn.gemm(M, K, K, Fn.op(a, 0, K, True), Fn.op(eye, 0, K, True), fo, K, pre_out=pre, act=Fn.ACT["gelu"],
                drop_p=0.1, seed=seed)
    f16 = Fn._act_dropout_cast16(pre, Fn.ACT["gelu"], 0.1, seed)
    assert torch.equal(f16, fo.to(torch.bfloat16))
    # fused output-dropout backward: bf16(dropout(dy) * scale) and its column sums
    dy = torch.randn(M, D, device="cuda")
    ref32 = torch.empty_like(dy)
    Fn._lib.call("b2p_dropout_scaled", dy.data_ptr(), ref32.data_ptr(), dy.numel(), 0.1, 77, 0.5, Fn._st())
    y16, cs = Fn._drop_cast_colsum(dy, 0.1, 77, 0.5, True)
    assert torch.equal(y16, ref32.to(torch.bfloat16))
    assert _rel(cs.cpu(), ref32.sum(0).cpu()) < 1e-5
    y16b, none = Fn._drop_cast_colsum(dy, 0.0, 0, 1.0, False)
    assert none is None and torch.equal(y16b, dy.to(torch.bfloat16))
    # GEMM epilogue writing C16 as fp16 (16-bit operands of both kinds)
    N = 192
    a16 = torch.randn(M, K, device="cuda").half()
    w16 = torch.randn(N, K, device="cuda").half()
    c32 = torch.empty(M, N, device="cuda")
    c16 = torch.empty(M, N, device="cuda", dtype=torch.float16)
    Fn.gemm(M, N, K, Fn.op(a16, 0, K, True), Fn.op(w16, 0, K, True), c32, N, C16=c16, c16_fp16=True)
    refm = a16.float() @ w16.float().t()
    assert _rel(c32.cpu(), refm.cpu()) < 1e-5
    assert torch.equal(c16, c32.half())


@pytest.mark.parametrize("B,T,D,dh", [(3, 100, 256, 64), (2, 249, 1024, 64), (1, 37, 512, 32), (2, 50, 256, 128),
                                      (1, 5, 256, 256)])
def test_layernorm_rotary_one_pass_bitwise(B, T, D, dh):
    """b2p_layernorm_rotary16 (LayerNorm + rotary, 16-bit outputs only) equals the two-launch form it
    replaces in the Conformer attention block -- LayerNorm with an fp32 output, then b2p_rotary16 of that
    output -- bit for bit, for the plain and rotated operands in fp16 and bf16, and its mean / rstd equal
    the LayerNorm kernel's."""
    Fn = _fn()
    torch.manual_seed(5)
    nh = D // dh
    x = 2 * torch.randn(B * T, D, device="cuda") + 0.3
    g, b = 1 + 0.1 * torch.randn(D, device="cuda"), 0.1 * torch.randn(D, device="cuda")
    cos_t, sin_t = Fn.rotary_tables(T, dh, 10000, "cuda")
    assert Fn.ln_rotary16_ok(D, dh)
    for half in (True, False):
        y, y16, mean, rstd, y16b = Fn._ln_fwd_x16(x, g, b, 1e-5, half, want_b16=True)
        r16 = Fn._rotary16(y, cos_t, sin_t, B, T, nh, dh, half)
        r16b = Fn._rotary16(y, cos_t, sin_t, B, T, nh, dh, False)
        h16, h16b, hr16, hr16b, m2, s2 = Fn._ln_rotary16(x, g, b, 1e-5, T, dh, cos_t, sin_t, half)
        torch.cuda.synchronize()
        assert h16.dtype == (torch.float16 if half else torch.bfloat16) and hr16b.dtype == torch.bfloat16
        assert torch.equal(m2, mean) and torch.equal(s2, rstd)
        assert torch.equal(h16, y16) and torch.equal(hr16, r16)
        assert torch.equal(h16b, y16b) and torch.equal(hr16b, r16b)


@pytest.mark.parametrize("act", [3, 1])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("NT,D,F", [(300, 128, 512), (7968, 1024, 4096)])
def test_ffn1_epilogue_bf16_copy_equals_recompute(act, p, NT, D, F):
    """The FFN1 GEMM's second 16-bit output (C16b: bf16(dropout(act(pre))) beside the fp16 forward
    operand) against the backward's recompute of the same operand from the fp32 pre-activation
    (b2p_act_dropout_cast16): bitwise equal, for SiLU (the Conformer) and GELU, with and without
    dropout, on the small-tile and the ping-pong kernels."""
    Fn = _fn()
    torch.manual_seed(5)
    h16 = torch.randn(NT, D, device="cuda").half()
    w1 = torch.randn(F, D, device="cuda") / math.sqrt(D)
    b1 = torch.randn(F, device="cuda") * 0.1
    pre = torch.empty(NT, F, device="cuda")
    f = torch.empty(NT, F, device="cuda", dtype=torch.float16)
    fb = torch.empty(NT, F, device="cuda", dtype=torch.bfloat16)
    seed = 1234 if p > 0 else 0
    with Fn.precision("bf16"), Fn.forward_f16(True):
        _, w1op = Fn._w_op16(w1, True)
        Fn.gemm(NT, F, D, Fn.op(h16, 0, D, True), w1op, None, F, bias=b1, pre_out=pre, act=act, drop_p=p, seed=seed,
                C16=f, c16_fp16=True, C16b=fb)
        ref = Fn._act_dropout_cast16(pre, act, p, seed)
    torch.cuda.synchronize()
    d = (fb.float() - ref.float()).abs()
    assert torch.equal(fb, ref), (int((d > 0).sum()), float(d.max()))


def test_conv_module_vector_paths_bitwise_equal_scalar_paths():
    """The float4 forms of the Conformer conv-module kernels (BatchNorm apply / backward passes, GLU,
    depthwise-conv LDS staging) against their scalar forms, which the library takes for operands that
    are not 16-B aligned: bitwise equal outputs (same per-element arithmetic)."""
    Fn = _fn()
    from wav2vec2forbrain_amd import _lib
    lib = _lib.load()
    P = Fn._p
    torch.manual_seed(11)
    B, T, C, K = 3, 150, 256, 31
    M = B * T

    def buf(n, fill=None):   # [16-B aligned, 4-B offset] views, one allocation each
        a, b = torch.empty(n + 4, device="cuda"), torch.empty(n + 4, device="cuda")
        if fill is not None:
            a[:n].copy_(fill)
            b[1:n + 1].copy_(fill)
        return a[:n], b[1:n + 1]

    st = Fn._st()
    x = torch.randn(M * C, device="cuda") * 2 + 0.3
    dy = torch.randn(M * C, device="cuda")
    a2 = torch.randn(M * 2 * C, device="cuda")
    gamma, beta = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    mean, rstd = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    w = torch.randn(C * K, device="cuda") * 0.2
    outs = []
    sums_ref = None
    for al in (0, 1):
        xs, dys, a2s = buf(M * C, x)[al], buf(M * C, dy)[al], buf(M * 2 * C, a2)[al]
        y, pre, g, dx, u, cv, dcv, du = (buf(M * C)[al] for _ in range(8))
        ws = torch.empty(int(lib.b2p_batchnorm_workspace(M, C)) + 4, device="cuda")
        sums = torch.empty(2 * C, device="cuda")
        _lib.call("b2p_batchnorm_apply", P(xs), P(mean), P(rstd), P(gamma), P(beta), P(y), P(pre), M, C, 3, st)
        _lib.call("b2p_batchnorm_bwd_sums", P(dys), P(pre), P(xs), P(mean), P(rstd), P(g), P(sums), P(sums, C), M, C, 3,
                  P(ws), st)
        # the column sums themselves take another reduction order on unaligned rows: dx from one set
        sums_ref = sums if sums_ref is None else sums_ref
        _lib.call("b2p_batchnorm_bwd_dx", P(g), P(xs), P(mean), P(rstd), P(gamma), P(sums_ref), P(sums_ref, C), P(dx), M,
                  C, M, st)
        _lib.call("b2p_glu_fwd", P(a2s), P(u), M, C, st)
        _lib.call("b2p_dwconv_fwd", P(u), P(w), P(cv), B, T, C, K, st)
        wsd = torch.empty(int(lib.b2p_dwconv_bwd_workspace(B, T, C, K)) + 4, device="cuda")
        ddw = torch.empty(C * K, device="cuda")
        _lib.call("b2p_dwconv_bwd", P(u), P(w), P(dys), P(du), P(ddw), B, T, C, K, P(wsd), st)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (y, pre, g, ws[:M * C], dx, u, cv, du, ddw)])
    names = ("bn y", "bn pre", "bn g", "bn g*xhat", "bn dx", "glu", "dwconv", "dwconv dx", "dwconv dw")
    for n, p, q in zip(names, outs[0], outs[1]):
        assert torch.equal(p, q), (n, float((p - q).abs().max()))


@pytest.mark.parametrize("M,N,batch,ld_pad,mode", [
    (7968, 1024, 1, 0, 0), (7968, 3 * 768, 1, 0, 0), (1000, 130, 1, 0, 0), (257, 64, 3, 0, 0),
    (5000, 300, 2, 3, 0), (4099, 96, 1, 0, 1), (3000, 200, 2, 0, 2), (2048, 1024, 1, 0, 3), (1, 5, 1, 0, 0),
    (1000, 130, 1, 1, 3), (999, 66, 2, 2, 2), (777, 40, 1, 1, 1)])
def test_colsum_one_launch(M, N, batch, ld_pad, mode):
    """Column sums in one launch (csrc/elementwise.hip colsum_fold*: the last-arriving row block of a
    column strip sums the strip's sc1 partials and resets its counter) against an fp64 torch sum:
    ragged M / N, batched, padded ld, every mode, accumulate, repeated launches (counter reuse), a
    captured graph replayed 3 times and two launches on concurrent streams."""
    from wav2vec2forbrain_amd import _lib
    Fn = _fn()
    torch.manual_seed(M + N)
    ld = N + ld_pad
    X = torch.randn(batch, M, ld, device="cuda") + 0.25
    Y = torch.randn(batch, M, ld, device="cuda")
    C = torch.randn(batch, N, device="cuda")
    Xd, Yd, Cd = X[..., :N].double(), Y[..., :N].double(), C.double()
    ref = {0: Xd.sum(1), 1: (Xd * Xd).sum(1), 2: (Xd * Yd).sum(1), 3: ((Xd - Cd[:, None, :]) ** 2).sum(1)}[mode]
    yarg = Y if mode == 2 else (C if mode == 3 else None)

    def run(out, acc=0, stream=None):
        ws = torch.empty(max(int(_lib.load().b2p_colsum_workspace(M, N)) * batch, 1), device="cuda")
        st = ctypes_stream(stream)
        _lib.call("b2p_colsum_batched", Fn._p(X), Fn._p(yarg), batch, M, N, ld, M * ld, mode, Fn._p(out), acc,
                  Fn._p(ws), st)
        return ws

    tol = 2e-6 * max(1.0, math.sqrt(M))
    outs = []
    for _ in range(3):
        o = torch.empty(batch, N, device="cuda")
        run(o)
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, outs[0])
        assert _rel(o.double(), ref) < tol
    o = outs[0].clone()
    run(o, acc=1)
    assert _rel(o.double(), 2 * ref) < tol
    # graph replay: the counters are reset by each launch's last block
    g = torch.cuda.CUDAGraph()
    og = torch.zeros(batch, N, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            keep = run(og)
    for _ in range(3):
        og.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(og, outs[0])
    del keep
    # two streams at once
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1, o2 = torch.empty(batch, N, device="cuda"), torch.empty(batch, N, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        k1 = run(o1, stream=s1)
    with torch.cuda.stream(s2):
        k2 = run(o2, stream=s2)
    torch.cuda.synchronize()
    assert torch.equal(o1, outs[0]) and torch.equal(o2, outs[0])
    del k1, k2


def ctypes_stream(stream=None):
    s = torch.cuda.current_stream() if stream is None else stream
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


def test_accum_rows_recs():
    """b2p_accum_rows_recs (csrc/adam.hip accum_rec_k): records {dst, src, numel, nrows, set} in one
    launch — plain accumulation (nrows 1), column sums of partial rows written (set) or accumulated,
    more records than one launch holds — against torch."""
    import ctypes
    from wav2vec2forbrain_amd import _lib
    torch.manual_seed(5)
    cases = [(1000, 1, 0), (4096, 125, 1), (768, 63, 0), (3, 7, 1), (1024, 32, 0)] * 14   # 70 records
    dsts, srcs, refs, recs = [], [], [], []
    for n, r, st in cases:
        d = torch.randn(n, device="cuda")
        s = torch.randn(r, n, device="cuda")
        refs.append((s.double().sum(0) + (0 if st else d.double())).float())
        dsts.append(d)
        srcs.append(s)
        recs += [d.data_ptr(), s.data_ptr(), n, r, st]
    arr = (ctypes.c_int64 * len(recs))(*recs)
    _lib.call("b2p_accum_rows_recs", arr, len(cases), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for d, ref in zip(dsts, refs):
        assert _rel(d, ref) < 1e-5


def test_colsum_pinned_counters_survive_pool_wrap():
    """Counter ranges of captured graphs stay reserved (b2p_colsum_pin_begin / _end / _unpin, as
    StepGraph.capture does): two captured graphs, then the allocation cursor moved to just before each
    graph's range so that the rotation wraps across them, then eager launches on a concurrent stream
    racing the replays of both graphs. Every result equals the fp64 sum; no eager launch was handed a
    reserved counter; unpinning frees the ranges."""
    import ctypes
    from wav2vec2forbrain_amd import _lib
    Fn = _fn()
    lib = _lib.load()
    torch.manual_seed(5)
    M, N, batch = 3000, 1000, 4
    X = torch.randn(batch, M, N, device="cuda") + 0.25
    ref = X.double().sum(1)

    def run(out, stream=None):
        ws = torch.empty(int(lib.b2p_colsum_workspace(M, N)) * batch, device="cuda")
        _lib.call("b2p_colsum_batched", Fn._p(X), None, batch, M, N, N, M * N, 0, Fn._p(out), 0, Fn._p(ws),
                  ctypes_stream(stream))
        return ws

    res = ctypes.c_int64()
    lib.b2p_colsum_pool_state(-1, ctypes.byref(res))
    reserved0 = res.value
    graphs, outs, keep, pins, starts = [], [], [], [], []
    s = torch.cuda.Stream()
    for _ in range(2):
        g = torch.cuda.CUDAGraph()
        o = torch.zeros(batch, N, device="cuda")
        s.wait_stream(torch.cuda.current_stream())
        starts.append(lib.b2p_colsum_pool_state(-1, None))
        _lib.check(lib.b2p_colsum_pin_begin(), "pin_begin")
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                keep.append(run(o))
        pins.append(lib.b2p_colsum_pin_end())
        graphs.append(g)
        outs.append(o)
    lib.b2p_colsum_pool_state(-1, ctypes.byref(res))
    assert res.value - reserved0 >= 2 * ((N + 127) // 128) * batch, res.value
    side = torch.cuda.Stream()
    for start in starts:
        lib.b2p_colsum_pool_state(start, None)        # the next eager range would overlap this graph's
        eager = [torch.empty(batch, N, device="cuda") for _ in range(4)]
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            ks = [run(e, stream=side) for e in eager]
        for g, o in zip(graphs, outs):
            o.zero_()
            g.replay()
        torch.cuda.synchronize()
        for o in outs + eager:
            assert _rel(o.double(), ref) < 2e-6 * math.sqrt(M)
        del ks
    for p in pins:
        lib.b2p_colsum_unpin(p)
    lib.b2p_colsum_pool_state(-1, ctypes.byref(res))
    assert res.value == reserved0, (res.value, reserved0)
    del keep


def test_batchnorm_16bit_outputs_bitwise():
    """b2p_batchnorm_fwd16 / b2p_batchnorm_apply16 (the Conformer conv module's BatchNorm + activation
    writing only the pointwise-conv-2 operands) against b2p_batchnorm_fwd / apply and a rounding of their
    fp32 output: equal bits for the fp16 and bf16 copies, the same statistics and pre-activation."""
    Fn = _fn()
    from wav2vec2forbrain_amd import _lib
    lib = _lib.load()
    P, st = Fn._p, Fn._st()
    torch.manual_seed(7)
    M, C = 1000, 512
    x = torch.randn(M, C, device="cuda") * 1.7 + 0.2
    gamma, beta = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
    ws = torch.empty(int(lib.b2p_batchnorm_workspace(M, C)), device="cuda")
    outs = {}
    for form in ("fp32", "16"):
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        y = torch.empty(M, C, device="cuda")
        y16 = torch.empty(M, C, device="cuda", dtype=torch.float16)
        y16b = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        pre, mean, rstd = torch.empty(M, C, device="cuda"), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        if form == "fp32":
            _lib.call("b2p_batchnorm_fwd", P(x), P(gamma), P(beta), P(rm), P(rv), P(y), P(pre), P(mean), P(rstd), M, C,
                      1e-5, 0.1, 3, P(ws), st)
        else:
            _lib.call("b2p_batchnorm_fwd16", P(x), P(gamma), P(beta), P(rm), P(rv), None, P(y16), 1, P(y16b), P(pre),
                      P(mean), P(rstd), M, C, 1e-5, 0.1, 3, P(ws), st)
        torch.cuda.synchronize()
        outs[form] = (y, y16, y16b, pre, mean, rstd, rm, rv)
    y, _, _, pre, mean, rstd, rm, rv = outs["fp32"]
    _, y16, y16b, pre2, mean2, rstd2, rm2, rv2 = outs["16"]
    assert torch.equal(y16, y.half()) and torch.equal(y16b, y.bfloat16())
    for a, b in ((pre, pre2), (mean, mean2), (rstd, rstd2), (rm, rm2), (rv, rv2)):
        assert torch.equal(a, b)
    # the SyncBN stage form: bf16 operand only
    yb = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
    _lib.call("b2p_batchnorm_apply16", P(x), P(mean), P(rstd), P(gamma), P(beta), None, P(yb), 0, None, None, M, C, 3,
              st)
    torch.cuda.synchronize()
    assert torch.equal(yb, y.bfloat16())


def test_conformer_conv_module_bn16_bitwise():
    """The conv module's 16-bit BatchNorm outputs (no fp32 activation, no cast passes) leave the tiny
    Conformer's bf16 training step bitwise unchanged: loss and every gradient."""
    Fn = _fn()
    from tests.helpers import CFG, batch_dict, build_model
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    cfg = CFG["tiny_conf"]
    b = batch_dict(cfg)
    batch = make_b2t_batch(b["x"], b["target"], b["day_idxs"], b["input_lens"], b["target_lens"]).cuda()
    res = []
    for on in (False, True):
        Fn._BN16[0] = on
        try:
            torch.manual_seed(0)
            Fn.SEEDS.reseed(1234)
            Fn.LD_SEEDS.reseed(1234)
            model = build_model(cfg)
            model.train()
            with Fn.precision("bf16"):
                out = model(batch)
                out.loss.backward()
                Fn.join_wgrad()
            torch.cuda.synchronize()
            res.append((float(out.loss), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}))
        finally:
            Fn._BN16[0] = True
    assert res[0][0] == res[1][0]
    assert res[0][1].keys() == res[1][1].keys()
    for n in res[0][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


def test_unfold_lens_and_ctc_targets_match_reference_expressions():
    """b2p_unfold_lens / b2p_ctc_targets (one launch each in the step) against the reference's own torch
    expressions on the same device tensors (src/model/b2p2t_model.py:170-173,
    src/model/w2v_custom_feat_extractor.py:70): bitwise, including lengths below the kernel size
    (negative quotients truncate toward zero) and targets at and below the blank."""
    Fn = _fn()
    g = torch.Generator().manual_seed(3)
    lens = torch.cat([torch.randint(-50, 5000, (997,), generator=g), torch.tensor([0, 1, 13, 14, 15, 16, 2 ** 24 + 3])])
    lens = lens.cuda()
    for k, s in ((14, 4), (32, 4), (1, 1), (7, 3)):
        ref = ((lens - k) / s).to(torch.int32)
        assert torch.equal(Fn.unfold_lens(lens, k, s), ref), (k, s)
    t = torch.randint(-5, 41, (32, 77), generator=g).cuda()
    assert torch.equal(Fn.ctc_targets(t), torch.where(t < 1, torch.tensor(-100, device="cuda"), t))
    assert torch.equal(Fn.ctc_targets(t[:, :5]), t[:, :5].masked_fill(t[:, :5] < 1, -100))   # non-contiguous view
