"""Autograd-visible operators of the b2p2t_gru+w2v training step, each a thin host wrapper over
the C ABI of libb2p_hip.so (include/b2p_hip.h). No operator here computes on the CPU or falls
back to a PyTorch kernel: tensors must be fp32 CUDA(HIP) tensors and every FLOP of the forward
and backward runs in the hand-written gfx950 kernels. PyTorch supplies device memory (caching
allocator), the stream and autograd bookkeeping only.

Operators (reference call sites in each docstring):
  front_end        Gaussian smoothing + day linear + softsign          (b2p2t_model.py:138-167)
  gru_layer        bidirectional GRU layer, optional implicit Unfold     (brain_feature_extractor.py:56-68)
  linear           nn.Linear (+ activation)                              (nn_helper.py:31-49, lm_head)
  dropout          nn.Dropout with a stateless, regenerable mask
  pos_conv_ln      pos-conv embedding + residual + LayerNorm + dropout   (TF Wav2Vec2Encoder.forward)
  encoder_layer    post-LN transformer layer                              (TF Wav2Vec2EncoderLayer)
  ctc_loss         log_softmax + CTCLoss(blank=0, mean, zero_infinity)   (w2v_custom_feat_extractor.py:81-90)
"""
from __future__ import annotations

import contextlib
import functools
import ctypes
import math
import threading
import weakref

import os

import torch

from . import _lib
from ._lib import GemmDesc, Operand, Epilogue

ACT = {"none": 0, None: 0, "gelu": 1, "softsign": 2, "silu": 3, "swish": 3}

class _State:
    # process-global (autograd runs backward on its own worker thread, so a thread-local
    # setting would not reach the backward GEMMs)
    prec = 0
    fwd16 = False   # forward_f16(): fp32-operand GEMMs of a forward pass on fp16 MFMA
    nosplit = False  # no split-K (deferred weight gradients issued on concurrent side streams)
    sync_bn = None   # process group for synchronised BatchNorm statistics (sync_batchnorm())
    gate = None      # LayerDrop gate (device int32) of the layer being issued in a captured step
    block = None     # error attribution: the B2P_FP32_OPS block whose forward is being issued
    x3forms = None   # x3_forms(): GEMM roles the bf16x3 mode runs single-pass / on two-term images


_state = _State()


@contextlib.contextmanager
def _gated(flag):
    """GEMM / fused-attention launches inside read the device LayerDrop flag (b2p_set_gate)."""
    old = _state.gate
    if flag is old:
        yield
        return
    _state.gate = flag
    _lib.call("b2p_set_gate", None if flag is None else flag.data_ptr())
    try:
        yield
    finally:
        _state.gate = old
        _lib.call("b2p_set_gate", None if old is None else old.data_ptr())


def _gate_aware(cls):
    """An encoder-layer autograd Function whose backward runs under the gate its forward ran under
    (a layer skipped by this replay's LayerDrop draw skips its backward GEMMs too)."""
    fwd, bwd = cls.forward, cls.backward

    @functools.wraps(fwd)
    def forward(ctx, *args):
        ctx.gate = _state.gate
        return fwd(ctx, *args)

    @functools.wraps(bwd)
    def backward(ctx, *grads):
        with _gated(ctx.gate):
            return bwd(ctx, *grads)

    cls.forward = staticmethod(forward)
    cls.backward = staticmethod(backward)
    return cls




PRECISION_MODES = {"bf16": 0, "fp32": 1, "bf16x3": 3}   # GemmDesc.precision of each mode's fp32-operand GEMMs


def _prec() -> int:
    return _state.prec


@contextlib.contextmanager
def precision(mode: str):
    """'bf16' (default: bf16 / fp16 MFMA, fp32 accumulate), 'fp32' (exact-fp32 MFMA parity mode) or
    'bf16x3' (the fp32 mode's operators with every GEMM on split-bf16 operands: hi*hi + hi*lo + lo*hi,
    ~16 significant bits per product, at a third of the bf16 MFMA rate instead of a sixteenth)."""
    old = _prec()
    _state.prec = PRECISION_MODES[mode]
    try:
        yield
    finally:
        _state.prec = old


@contextlib.contextmanager
def forward_f16(on: bool = True):
    """In bf16 mode, run the fp32-operand GEMMs issued inside (a model's forward) on fp16 MFMA:
    operands rounded to 11 significant bits instead of 8, same MFMA rate. The 24-layer Conformer's
    CTC loss is biased by the rounding noise of its logits (the loss is convex in them), +1.5e-3
    relative at bf16; fp16 forward operands cut that noise ~64x in variance.
    Backward GEMMs (outside the context) stay bf16: gradients span magnitudes below fp16's range."""
    old = _state.fwd16
    _state.fwd16 = bool(on)
    try:
        yield
    finally:
        _state.fwd16 = old


# error attribution (tools/bf16_err.py): blocks listed in B2P_FP32_OPS run their forward in exact fp32
_FP32_OPS = set(filter(None, os.environ.get("B2P_FP32_OPS", "").split(",")))
# error attribution (tools/traj_err_ft.py): named precision switches of a diagnostic run
DIAG_SWITCHES: set = set(filter(None, os.environ.get("B2P_DIAG", "").split(",")))


@contextlib.contextmanager
def _fp32_if(name: str):
    old = _state.block
    _state.block = name
    try:
        if name in _FP32_OPS:
            with precision("fp32"):
                yield
        else:
            yield
    finally:
        _state.block = old


# error attribution (tools/traj_err.py): with B2P_FP32_BWD=1 a block's backward runs in the precision
# its forward ran in, so B2P_FP32_OPS=<block> puts that block's forward AND backward in exact fp32
_BWD_FOLLOWS_FWD = [os.environ.get("B2P_FP32_BWD", "0") == "1"]
_FP32_BWD_OPS: set = set()   # blocks whose backward follows their forward's precision regardless
_FP32_BWD_ONLY: set = set()  # blocks whose backward runs in exact fp32 (forward unchanged)
# blocks whose backward always runs in the precision their forward ran in: the GRU layer, whose bf16-mode
# forward (persistent recurrences, lane-native saved state) only its bf16-mode backward can consume
_BWD_FOLLOWS_BLOCKS = frozenset({"gru"})


def _prec_follow(cls):
    fwd, bwd = cls.forward, cls.backward

    @functools.wraps(fwd)
    def forward(ctx, *args):
        ctx.prec_fwd = _state.prec
        ctx.block = _state.block
        return fwd(ctx, *args)

    @functools.wraps(bwd)
    def backward(ctx, *grads):
        if "bwd32path" in DIAG_SWITCHES:   # diagnostic: fp32-operand backward, GEMMs rounding to fp16 / bf16
            with forward_f16("bwdf16" in DIAG_SWITCHES):
                return bwd(ctx, *grads)
        if ctx.block in _FP32_BWD_ONLY and _state.prec != 1:
            with precision("fp32"):
                return bwd(ctx, *grads)
        if (_BWD_FOLLOWS_FWD[0] or ctx.block in _FP32_BWD_OPS or ctx.block in _BWD_FOLLOWS_BLOCKS) \
                and ctx.prec_fwd != _state.prec:
            with precision({v: k for k, v in PRECISION_MODES.items()}[ctx.prec_fwd]):
                return bwd(ctx, *grads)
        return bwd(ctx, *grads)

    cls.forward = staticmethod(forward)
    cls.backward = staticmethod(backward)
    return cls


# -------------------------------------------------------------------------------------------
# Deferred gradients of FROZEN parameters (reference semantics: the frozen w2v still gets weight
# gradients accumulated into .grad every step, src/train/train_loop.py:44,66 — they feed nothing
# in the step). Their GEMMs are queued during the encoder backward and flushed onto a side stream
# when the (4-CU) GRU recurrence backward starts, so they fill the otherwise idle chip; they
# accumulate into p.grad in the GEMM epilogue (beta = 1) instead of autograd's separate add.
# join_wgrad() orders the side stream back into the main stream (train step, optimizer).
_DIAG_SKIP_ACC = os.environ.get("B2P_DIAG_SKIP_SMALL_ACC") == "1"   # diagnostic only
# diagnostic only (never a bench setting): drop the queued frozen weight-gradient launches, to measure how
# much of the step's tail the side stream holds
_DIAG_SKIP_WGRAD = os.environ.get("B2P_DIAG_SKIP_WGRAD") == "1"
# workgroups a 128 x 128 split-K GEMM aims for (the split count is capped at one slice per 1024 of K)
_SPLITK_WGS = int(os.environ.get("B2P_SPLITK_WGS", "512"))
_PP_SPLIT = os.environ.get("B2P_PP_SPLIT", "0") == "1"   # every eligible split-K GEMM on the ping-pong kernel
# split-K GEMMs with at least this many outputs go to the 256 x 256 ping-pong kernel: the Conformer's
# frozen weight gradients (4096 x 1024, 3072 x 1024; K = 7968 tokens) -8.6 ms per step; the base
# model's (768 x 3072 and smaller) measured 0.2 ms slower on it, so they stay on the 128 x 128 split
_PP_MIN_MN = int(os.environ.get("B2P_PP_MIN_MN", str(3 * 1024 * 1024)))
# ... and only while the unsplit 128 x 128 grid has fewer tiles than this (a grid that fills the chip by
# itself needs no fp32 slabs and no reduce pass): the Conformer's 7968 x 1024 backward-data GEMMs (504
# tiles) 69.73 -> 68.54 ms per step unsplit; the base model's 7968 x 768 (378 tiles, 1.5 rounds of the
# CUs) stay split (14.99 vs 15.13 ms unsplit), profiles/r05o_pp_split_rule_ab.txt
_PP_SPLIT_MAX_BLOCKS = int(os.environ.get("B2P_PP_SPLIT_MAX_BLOCKS", "448"))
# ... unless K is long enough that one 128 x 128 tile's K loop dominates (the front end's implicit-unfold
# backward-data GEMM, 8192 x 1024 x 24576 in the Conformer step: 1.39 ms unsplit on 128 x 128 tiles)
_PP_SPLIT_LONG_K = int(os.environ.get("B2P_PP_SPLIT_LONG_K", "8192"))


class _Deferred:
    ids: set = set()
    queue: list = []          # (fn, tensors used, key = id of the parameter it updates)
    accs: list = []           # (parameter, small gradient) pairs accumulated in one launch
    sides: list = []          # side streams (B2P_SIDE_STREAMS, default 1: several concurrent weight-
                              # gradient streams starved the main stream, 15.1 -> 17.2-18.8 ms/step)
    lane: dict = {}           # parameter id -> side stream index (fixed: one stream per parameter)
    pending = False
    split = os.environ.get("B2P_DEFER_SPLIT", "1") == "1"   # split-K for the deferred GEMMs


def set_deferred_wgrad(params, names=None) -> None:
    """Parameters whose gradients may be deferred (frozen: not optimised, not all-reduced). names
    (optional, {id(p): qualified name}): the layer-independent role of each parameter (the name with its
    layer indices masked), which sizes the batched weight-gradient slot buffers (_Home) by the number of
    layers that hold a parameter of that role, not by every frozen parameter of the same shape."""
    import re
    _Deferred.ids = {id(p) for p in params if p is not None}
    # frozen parameters by storage address: their staged 16-bit GEMM operand copies are cached
    # (keyed by the tensor version, so an in-place load still invalidates them)
    _CAST_CACHE.clear()
    _FROZEN_PTR.clear()
    _FROZEN_PTR.update({p.data_ptr(): p for p in params if p is not None and p.is_cuda})
    _FROZEN_ROLE.clear()
    if names:
        _FROZEN_ROLE.update({id(p): re.sub(r"\.\d+\.", ".#.", names[id(p)]) for p in params
                             if p is not None and id(p) in names})
    _HOMES.clear()


def deferred_wgrad_active() -> bool:
    """Some parameter's gradient work is deferred to the side streams (set_deferred_wgrad)."""
    return bool(_Deferred.ids)


def _defer_ok(p) -> bool:
    return p is not None and id(p) in _Deferred.ids


def _acc_param(p, g) -> None:
    if p.grad is None:
        p.grad = g
    else:
        p.grad.add_(g)


def _defer_acc(p, g) -> None:
    """Accumulate a ready gradient tensor into p.grad on the side stream (all of a flush's small
    accumulations go out as ONE multi-tensor launch, b2p_accum_recs)."""
    if _DIAG_SKIP_ACC:
        return
    if not _LAZY_COLSUM:
        g = _mat(g)
    _Deferred.accs.append((p, g))


def _defer_small(prms, grads):
    """Small gradients of frozen parameters (LayerNorm / bias / BatchNorm / depthwise taps) queued for
    the side stream's one multi-tensor accumulation instead of one autograd add launch each; the
    returned list has None where a gradient was taken over."""
    out = list(grads)
    for k, (p, g) in enumerate(zip(prms, grads)):
        if g is not None and _defer_ok(p):
            _defer_acc(p, g)
            out[k] = None
        else:
            out[k] = _mat(g)
    return out


def _flush_accs(sd) -> None:
    """The queued small-gradient accumulations on side stream sd: a parameter without .grad takes
    the tensor itself, the rest are batched into b2p_accum_rows_recs records {p.grad, g, numel}. The
    records of one launch run in parallel (one per blockIdx.y), so a destination appears at most once
    per launch: a parameter queued twice in one flush goes into the next launch, after the first."""
    recs, n, dsts = [], 0, set()

    def launch():
        nonlocal recs, n
        if n:
            arr = (ctypes.c_int64 * len(recs))(*recs)
            _lib.call("b2p_accum_rows_recs", arr, n, _st())
        recs, n = [], 0
        dsts.clear()

    with torch.cuda.stream(sd):
        for p, g in _Deferred.accs:
            if p.grad is not None and p.grad.data_ptr() in dsts:
                launch()
            if isinstance(g, ColsumParts):   # partial rows: summed (and accumulated) in the batched launch
                parts = g.parts
                parts.record_stream(sd)
                ok = (p.grad is None or (p.grad.is_contiguous() and p.grad.dtype == torch.float32
                                          and p.grad.numel() == parts.shape[1]))
                if not ok:
                    p.grad.add_(g.materialize().view_as(p.grad))
                    continue
                st = p.grad is None
                if st:
                    p.grad = torch.empty(p.shape, device=parts.device)
                recs += [p.grad.data_ptr(), parts.data_ptr(), parts.shape[1], parts.shape[0], int(st)]
                dsts.add(p.grad.data_ptr())
                n += 1
                continue
            g.record_stream(sd)
            if p.grad is None:
                p.grad = g
            elif (p.grad.is_contiguous() and g.is_contiguous() and p.grad.dtype == g.dtype == torch.float32
                  and p.grad.numel() == g.numel() and p.grad.device == g.device):
                recs += [p.grad.data_ptr(), g.data_ptr(), g.numel(), 1, 0]
                dsts.add(p.grad.data_ptr())
                n += 1
            else:
                p.grad.add_(g)
        launch()
    _Deferred.accs.clear()


def _gate_wrap(run):
    """A deferred launch keeps the LayerDrop gate of the layer that queued it."""
    gate = _state.gate
    if gate is None:
        return run

    def gated():
        with _gated(gate):
            run()
    return gated


def _defer_wgemm_rows(ps, fn, *tensors) -> None:
    """Like _defer_wgemm for parameters whose gradients are row blocks of ONE GEMM output (Q, K, V
    weights of the fused QKV projection): their .grad are views of one buffer, so a single GEMM
    writes or accumulates all of them."""
    prec = _prec()

    def run():
        old = _state.prec
        _state.prec = prec
        try:
            rows = [p.shape[0] for p in ps]
            g0 = ps[0].grad
            fused = g0 is not None and all(p.grad is not None for p in ps)
            if fused:
                base = g0.untyped_storage().data_ptr()
                off = g0.storage_offset()
                for p in ps:
                    fused = fused and p.grad.is_contiguous() and p.grad.untyped_storage().data_ptr() == base \
                        and p.grad.storage_offset() == off
                    off += p.numel()
            if fused:
                buf = torch.as_strided(g0, (sum(rows),) + tuple(ps[0].shape[1:]), g0.stride())
                fn(buf, 1.0)
            elif all(p.grad is None for p in ps):
                buf = torch.empty((sum(rows),) + tuple(ps[0].shape[1:]), device=ps[0].device)
                fn(buf, 0.0)
                r = 0
                for p, n in zip(ps, rows):
                    p.grad = buf[r:r + n]
                    r += n
            else:   # mixed state: compute, then accumulate per parameter
                buf = torch.empty((sum(rows),) + tuple(ps[0].shape[1:]), device=ps[0].device)
                fn(buf, 0.0)
                r = 0
                for p, n in zip(ps, rows):
                    _acc_param(p, buf[r:r + n])
                    r += n
        finally:
            _state.prec = old
    _Deferred.queue.append((_gate_wrap(run), tensors, id(ps[0]), None))


def _defer_bias_rows(ps, x, M, N) -> bool:
    """The column sums of x (M x N fp32, N = the concatenated lengths of the bias vectors ps) as the
    gradients of frozen biases: queued for the side stream (the same b2p_colsum launch, accumulating into
    their .grad) instead of run on the main stream. False when a bias is not a deferred frozen one."""
    if not (_LAZY_COLSUM and all(_defer_ok(q) for q in ps)):
        return False
    _defer_wgemm_rows(ps, lambda out, beta: colsum(x, M, N, out, accumulate=beta == 1.0), x)
    return True


def _defer_dwconv_wgrad(w, u, dc, B, T, D, K) -> None:
    """The depthwise-conv weight gradient of a frozen Conformer conv module (b2p_dwconv_bwd with no input
    gradient: tile partials, their column sum, the [C][K] transpose) queued for the side stream; the
    result joins the flush's batched accumulation into w.grad."""
    def run():
        ws = torch.empty(int(_lib.load().b2p_dwconv_bwd_workspace(B, T, D, K)), device=u.device)
        g = torch.empty_like(w)
        _lib.call("b2p_dwconv_bwd", _p(u), _p(w), _p(dc), None, _p(g), B, T, D, K, _p(ws), _st())
        _defer_acc(w, g)
    _Deferred.queue.append((_gate_wrap(run), (u, dc), id(w), None))


def _defer_wgemm(p, fn, *tensors) -> None:
    """Queue fn(out, beta): a weight-gradient GEMM writing (beta 0) or accumulating (beta 1) p.grad."""
    prec = _prec()

    def run():
        old = _state.prec
        _state.prec = prec
        try:
            if p.grad is None:
                p.grad = torch.empty_like(p)
                fn(p.grad, 0.0)
            else:
                fn(p.grad, 1.0)
        finally:
            _state.prec = old
    _Deferred.queue.append((_gate_wrap(run), tensors, id(p), None))


class _WSpec:
    """A deferred frozen weight gradient dW[M][N] = a[:, a_off:a_off+M]^T b (K = tokens, both 16-bit
    operands m/n-contiguous): ps are the parameters whose .grad are consecutive row blocks of dW."""
    __slots__ = ("ps", "M", "N", "K", "a", "a_off", "lda", "b", "ldb", "gate", "prec")

    def __init__(self, ps, M, N, K, a, a_off, lda, b, ldb):
        self.ps, self.M, self.N, self.K = tuple(ps), M, N, K
        self.a, self.a_off, self.lda, self.b, self.ldb = a, a_off, lda, b, ldb
        self.gate, self.prec = _state.gate, _prec()

    def key(self):
        # parameters by (rows, numel), not shape: a Conformer's out-projection weight (D, D) and its
        # pointwise conv-2 weight (D, D, 1) share one batched launch (two 1.5-round grids -> one of 3)
        return (self.M, self.N, self.K, self.lda, self.ldb, self.a.dtype, self.b.dtype, self.prec,
                tuple(_pkey(p) for p in self.ps))


# B2P_WGRAD_MERGE=1: batch groups keyed by (rows, numel) per parameter instead of the full shapes (measured
# neutral on Conformer-large: 64.93 / 65.12 vs 65.14 / 65.06 ms, profiles/r05aw_wgrad_merge_ab.txt)
_WGRAD_MERGE = os.environ.get("B2P_WGRAD_MERGE", "0") == "1"


def _pkey(p):
    return (p.shape[0], p.numel()) if _WGRAD_MERGE else tuple(p.shape)


# B2P_WGRAD_BATCH=0: every deferred frozen weight gradient is its own (split-K) launch
_WGRAD_BATCH = [os.environ.get("B2P_WGRAD_BATCH", "1") != "0"]


def _defer_wspec(ps, M, N, K, a, a_off, lda, b, ldb) -> None:
    """Queue a frozen weight gradient as a spec: flush_wgrad batches the same-shape gradients of all
    layers into one launch (nz1 = layers, the operands gathered per layer, the gradients as views of one
    buffer, a LayerDrop gate per layer); a lone spec runs as the single launch below."""
    spec = _WSpec(ps, M, N, K, a, a_off, lda, b, ldb)
    fn = lambda o, bt: gemm(M, N, K, op(a, a_off, lda, False), op(b, 0, ldb, False), o, N, beta=bt)
    if len(ps) == 1:
        _defer_wgemm(ps[0], fn, a, b)
    else:
        _defer_wgemm_rows(ps, fn, a, b)
    fn_, ts, key, _ = _Deferred.queue[-1]
    _Deferred.queue[-1] = (fn_, ts, key, spec)


def _i64_dev(vals, dev):
    """A device int64 tensor holding vals, written by a kernel launch (graph-capturable)."""
    t = torch.empty(len(vals), dtype=torch.int64, device=dev)
    arr = (ctypes.c_int64 * len(vals))(*vals)
    _lib.call("b2p_i64_fill", _p(t), arr, len(vals), _st())
    return t


def _gathered_op(ts, offs, ld, dtype):
    """One m/n-contiguous 16-bit Operand over several tensors: base = the lowest address, member z1 at
    gather1[z1] * 8 elements (every address 16-byte aligned)."""
    addrs = [t.data_ptr() + 2 * o for t, o in zip(ts, offs)]
    base = min(addrs)
    if any((x - base) % 16 for x in addrs):
        return None, None
    idx = _i64_dev([(x - base) // 16 for x in addrs], ts[0].device)
    o = Operand()
    o.ptr = base
    o.ld = ld
    o.bs1, o.bs2 = 8, 0
    o.gather1 = idx.data_ptr()
    o.inner_is_k = 0
    o.conv = 0
    o.dtype = 1 if dtype == BF16 else 2
    return o, idx


_WGRAD_DEBUG = os.environ.get("B2P_WGRAD_DEBUG") == "1"


def _wdbg(msg, specs):
    if _WGRAD_DEBUG:
        s0 = specs[0]
        print(f"wgrad batch {s0.M}x{s0.N}x{s0.K} x{len(specs)}: {msg}", flush=True)


class _Home:
    """The gradients of every frozen parameter (tuple) of one weight-gradient shape as slots of one
    zero-initialised buffer [slots][M][N], sized for the layers of the roles that use it (it grows only
    outside captures, so a captured step can rely on it): p.grad is a view of its slot, and any subset
    of the layers (LayerDrop skips some in eager steps) is one batched launch over the slots, the
    absent members under a closed gate."""

    def __init__(self, M, N, cap, dev):
        self.M, self.N = M, N
        self.buf = torch.zeros(cap, M, N, device=dev)
        self.slot = {}        # tuple of parameter ids -> slot
        self.members = []     # slot -> tuple of parameters
        self.dirty = []       # slot -> its memory may hold a value (it was bound once)

    def grow(self, cap) -> None:
        """A bigger buffer (outside captures only): the slots' values move over and every member's p.grad
        that was a slot view becomes the view of its new slot (a captured step never sees the old one:
        homes grow in eager steps, which precede every capture of the shape)."""
        old = self.buf
        self.buf = torch.zeros(cap, self.M, self.N, device=old.device)
        self.buf[:old.shape[0]].copy_(old)
        for i, ps in enumerate(self.members):
            r = 0
            for p in ps:
                ov = old[i, r:r + p.shape[0]].view(p.shape)
                if p.grad is not None and p.grad.data_ptr() == ov.data_ptr():
                    p.grad = self.view(i, p, r)
                r += p.shape[0]

    def ensure(self, ps):
        k = tuple(id(p) for p in ps)
        i = self.slot.get(k)
        if i is None:
            if len(self.members) >= self.buf.shape[0]:
                return None
            i = self.slot[k] = len(self.members)
            self.members.append(tuple(ps))
            self.dirty.append(False)
        return i

    def view(self, i, p, r):
        return self.buf[i, r:r + p.shape[0]].view(p.shape)

    def bindable(self, i, ps) -> bool:
        """Binding slot i needs no zero / copy pass (what a captured step may not contain)."""
        r = 0
        for p in ps:
            g = p.grad
            if g is None and self.dirty[i]:
                return False
            if g is not None and g.data_ptr() != self.view(i, p, r).data_ptr():
                return False
            r += p.shape[0]
        return True

    def bind(self, i, ps) -> None:
        """p.grad of every parameter of slot i becomes its slot view: a None gradient starts from a zeroed
        slot, a gradient held elsewhere is moved in."""
        r = 0
        for p in ps:
            v = self.view(i, p, r)
            g = p.grad
            if g is None:
                if self.dirty[i]:
                    v.zero_()
                p.grad = v
            elif g.data_ptr() != v.data_ptr() or g.stride() != v.stride():
                v.copy_(g)
                p.grad = v
            r += p.shape[0]
        self.dirty[i] = True


_HOMES: dict = {}
# same-shape groups of frozen weight gradients that could not run as one batched launch (no slot, unaligned
# operands) and ran one launch per gradient instead: a slow path the tests require to stay unused
WGRAD_FALLBACKS = [0]
_ZERO_GATE: dict = {}   # device -> int32 0 (a closed LayerDrop gate for absent batch members)


def _zero_gate(dev):
    z = _ZERO_GATE.get(str(dev))
    if z is None:
        z = _ZERO_GATE[str(dev)] = torch.zeros(1, dtype=torch.int32, device=dev)
    return z


def _run_wspecs(specs) -> bool:
    """Batched launches for same-shape frozen weight-gradient specs (on the current side stream), over
    the slots of their _Home: the members present accumulate (beta 1) into their slot views, the slots
    of absent layers run under a closed gate (their K loop skipped, += 0). False when the operands do
    not allow a gathered view (the caller then runs the specs one by one)."""
    s0 = specs[0]
    M, N, K = s0.M, s0.N, s0.K
    dev = s0.a.device
    key = s0.key()[:2] + s0.key()[3:]   # the group key without K (the tokens of this batch shape)
    home = _HOMES.get(key)
    cap = capturing()
    if home is None:
        if cap:   # a home is allocated (zeroed) outside captures only
            _wdbg("no home before the capture", specs)
            return False
        # slots: one per layer holding a role that leads a slot of this shape (the roles of the specs'
        # first parameters; the Conformer's ffn1 / ffn2 share a home, Wq / Wk / Wv / Wo share a shape but
        # not a home; a role first met in a later eager step grows the home); without roles every frozen
        # parameter of the shape counts, divided over a slot's members
        shape0 = _pkey(s0.ps[0])
        roles = {_FROZEN_ROLE.get(id(sp.ps[0])) for sp in specs}
        if None not in roles:
            nslots = sum(1 for q in _FROZEN_PTR.values() if _pkey(q) == shape0 and _FROZEN_ROLE.get(id(q)) in roles)
        else:
            nslots = -(-sum(1 for q in _FROZEN_PTR.values() if _pkey(q) == shape0) // len(s0.ps))
        home = _HOMES[key] = _Home(M, N, max(1, nslots), dev)
    if not cap:   # members new to the home beyond its capacity: grow it once (eager steps only)
        new = {tuple(id(p) for p in sp.ps) for sp in specs} - set(home.slot)
        if len(home.members) + len(new) > home.buf.shape[0]:
            home.grow(len(home.members) + len(new))
    at = {}
    for sp in specs:
        i = home.ensure(sp.ps)
        if i is None or (cap and not home.bindable(i, sp.ps)):
            _wdbg("slot unavailable", specs)
            return False
        at[i] = sp
    for i, sp in at.items():
        home.bind(i, sp.ps)
    nslot = len(home.members)
    # every chunk's gathered operands first: a chunk that cannot be gathered (operands not 16-byte
    # aligned) makes the caller run ALL the specs one by one, so nothing may have been launched yet
    # only the span of slots that holds present members (slots of layers absent from this flush would
    # run gated, += 0)
    lo, hi = min(at), max(at) + 1
    chunks = []
    for c0 in range(lo, hi, 64):
        c1 = min(hi, c0 + 64)
        mem = [at.get(i) for i in range(c0, c1)]
        if all(m is None for m in mem):
            continue
        fill = next(m for m in mem if m is not None)
        A, ia = _gathered_op([(m or fill).a for m in mem], [(m or fill).a_off for m in mem], s0.lda, s0.a.dtype)
        B, ib = _gathered_op([(m or fill).b for m in mem], [0] * len(mem), s0.ldb, s0.b.dtype)
        if A is None or B is None:
            _wdbg("operands not 16-byte aligned", specs)
            return False
        chunks.append((c0, c1, mem, A, ia, B, ib))
    old_prec, old_split = _state.prec, _state.nosplit
    _state.prec = s0.prec
    try:
        for c0, c1, mem, A, ia, B, ib in chunks:
            n = c1 - c0
            zg = _zero_gate(dev)
            gates = [zg if m is None else m.gate for m in mem]
            gp = (_i64_dev([0 if g is None else g.data_ptr() for g in gates], dev)
                  if any(g is not None for g in gates) else None)
            # the members' tiles fill the chip: no K split (no fp32 slabs, no reduce pass)
            _state.nosplit = old_split or -(-M // 128) * -(-N // 128) * n >= 256
            with _gated(None):
                if gp is not None:
                    _lib.call("b2p_set_gate_batch", gp.data_ptr())
                try:
                    gemm(M, N, K, A, B, home.buf[c0], N, cbs1=M * N, nz1=n, beta=1.0)
                finally:
                    if gp is not None:
                        _lib.call("b2p_set_gate_batch", None)
            del gp
            _wdbg(f"batched slots {c0}..{c1} ({sum(m is not None for m in mem)} present)", specs)
        del chunks
    finally:
        _state.prec, _state.nosplit = old_prec, old_split
    return True


def flush_wgrad(after=None) -> None:
    """Launch the queued frozen-parameter gradient work on the side streams, ordered after the event
    `after` (recorded by the caller before a long kernel it wants to run beside) or after everything
    the main stream has queued so far. Each parameter's work always goes to the same side stream
    (its accumulations stay ordered); independent weight-gradient GEMMs on different streams run
    concurrently, which fills the chip without split-K partial sums and their reduce launches."""
    if _WGRAD_DEBUG:
        print(f"flush_wgrad: {len(_Deferred.queue)} queued, {len(_Deferred.accs)} accs, after={after is not None}, "
              f"capturing={capturing()}", flush=True)
    if _DIAG_SKIP_WGRAD:
        _Deferred.queue.clear()
    if not _Deferred.queue and not _Deferred.accs:
        return
    main = torch.cuda.current_stream()
    if not _Deferred.sides:
        n = max(1, int(os.environ.get("B2P_SIDE_STREAMS", "1")))
        _Deferred.sides = [torch.cuda.Stream(device=main.device) for _ in range(n)]
    sides = [main] if SERIAL_SIDE else _Deferred.sides
    for sd in sides:
        if after is not None:
            sd.wait_event(after)
        else:
            sd.wait_stream(main)
    old = _state.nosplit
    _state.nosplit = not _Deferred.split
    try:
        # same-shape frozen weight gradients of the layers: one batched launch per shape (one side
        # stream keeps every parameter's work on one stream, as the lanes below do)
        batch = _WGRAD_BATCH[0] and len(sides) == 1
        groups, order = {}, []
        for ent in _Deferred.queue:
            spec = ent[3]
            if batch and spec is not None:
                k = spec.key()
                if k not in groups:
                    groups[k] = []
                    order.append(("g", k))
                groups[k].append(ent)
            else:
                order.append(("s", ent))
        for kind, x in order:
            ents = groups[x] if kind == "g" else [x]
            sd = sides[_Deferred.lane.setdefault(ents[0][2], len(_Deferred.lane) % len(sides))]
            with torch.cuda.stream(sd):
                batched = kind == "g" and _run_wspecs([e[3] for e in ents])
                if kind == "g" and not batched:
                    WGRAD_FALLBACKS[0] += 1
                if not batched:
                    for fn, _, key, _ in ents:
                        with torch.cuda.stream(sides[_Deferred.lane.setdefault(key, len(_Deferred.lane) % len(sides))]):
                            fn()
            for _, ts, key, _ in ents:
                for t in ts:
                    t.record_stream(sd if kind == "g" else sides[_Deferred.lane[key]])
        if _Deferred.accs:
            _flush_accs(sides[0])
    finally:
        _state.nosplit = old
    _Deferred.queue.clear()
    _Deferred.pending = True


# B2P_SERIAL_SIDE=1 (measurement only: PMC censuses, whose per-dispatch counters would otherwise mix the
# concurrent side-stream kernels' bytes into the main stream's): the side-stream work runs on the main
# stream, in issue order
SERIAL_SIDE = os.environ.get("B2P_SERIAL_SIDE", "0") == "1"


def _join_sides() -> None:
    """The current stream waits for the work already flushed to the side streams (the queue stays)."""
    if _Deferred.pending:
        cur = torch.cuda.current_stream()
        for sd in _Deferred.sides:
            cur.wait_stream(sd)
        _Deferred.pending = False


def join_wgrad() -> None:
    """Flush, then make the current stream wait for the side streams."""
    flush_wgrad()
    _join_sides()


class _Segments:
    """The segmented capture in progress (train/step_graph.py _SegmentedCapture) and, while a replay
    runs the host calls between its segments, how many segments follow the current call."""
    active = None
    remaining = 0


def collective(fn) -> None:
    """A host-issued collective (a torch.distributed call) at this point of the step. Eager: fn()
    now. Inside a segmented capture: the captured segment ends here (its side-stream forks joined, as
    a graph requires), and every replay calls fn() between this segment and the next — a collective is
    never captured, the segments around it are."""
    seg = _Segments.active
    if seg is None:
        fn()
        return
    _join_sides()
    if _KEEP_PLAN[0] is not None:
        _KEEP_PLAN[0].join()
    seg.split(fn)


def segments_remaining() -> int:
    """Inside a host call between the segments of a replayed step: the segments still to run."""
    return _Segments.remaining


def set_precision(mode: str) -> None:
    _state.prec = PRECISION_MODES[mode]


_GEMM_TIMING = [0]


def set_gemm_timing(on: bool) -> None:
    """Tag every GEMM launch for HIP-event timing (bench.py roofline; b2p_timing_enable first)."""
    _GEMM_TIMING[0] = _lib.TIMING_GEMM if on else 0


# ------------------------------------------------------------------ dropout seeds
class _SeedStream:
    """64-bit seeds for the stateless dropout masks, drawn from a CPU generator so that a run is
    reproducible from torch.manual_seed (the reference seeds torch at src/experiments/experiment.py:34)."""

    def __init__(self):
        self.gen = None

    def next(self) -> int:
        if self.gen is None:
            self.gen = torch.Generator()
            self.gen.manual_seed(torch.initial_seed() & 0xFFFFFFFFFFFF)
        return int(torch.randint(0, 2 ** 62, (1,), generator=self.gen).item())

    def reseed(self, seed: int) -> None:
        self.gen = torch.Generator()
        self.gen.manual_seed(seed)


SEEDS = _SeedStream()
# the device LayerDrop draws of captured steps: a stream of its own that is NOT offset by the rank (the
# reference skips a layer for the whole batch, and every rank's host draw in eager steps comes from
# the equal host torch seed), so replayed data-parallel steps drop the same layers on every rank
LD_SEEDS = _SeedStream()


def _chk(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{name}: expected a HIP device tensor (the product path has no CPU fallback)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name}: expected a contiguous tensor")


def _p(t, off: int = 0):
    if t is None:
        return None
    es = t.element_size() if isinstance(t, torch.Tensor) else 4
    return t.data_ptr() + es * off


def _st():
    return _lib.stream_ptr()


# ------------------------------------------------------------------ GEMM plumbing
def op(t, off=0, ld=0, k_inner=True, bs1=0, bs2=0, gather=None):
    o = Operand()
    o.ptr = _p(t, off)
    o.ld = ld
    o.bs1 = bs1
    o.bs2 = bs2
    o.gather1 = None if gather is None else gather.data_ptr()
    o.inner_is_k = 1 if k_inner else 0
    o.conv = 0
    o.dtype = 0
    if isinstance(t, torch.Tensor):
        o.dtype = 1 if t.dtype == torch.bfloat16 else (2 if t.dtype == torch.float16 else 0)
    return o


def conv_op(t, off, ld, T_out, T_in, stride, pad, Cg, sample_stride, k_inner=True, bs1=0, bs2=0):
    o = op(t, off, ld, k_inner, bs1, bs2)
    o.conv = 1
    o.conv_T_out = T_out
    o.conv_T_in = T_in
    o.conv_stride = stride
    o.conv_pad = pad
    o.conv_Cg = Cg
    o.conv_sample_stride = sample_stride
    return o


def gemm(M, N, K, A: Operand, B: Operand, C, ldc, c_off=0, cbs1=0, cbs2=0, nz1=1, nz2=1, alpha=1.0,
         beta=0.0, bias=None, biasbs1=0, bias_gather=None, pre_out=None, act=0, act_bwd=0, aux=None, ldaux=0, abs1=0, abs2=0,
         drop_p=0.0, seed=0, residual=None, r_off=0, ldr=0, rbs1=0, rbs2=0, timing=0, C16=None, pre16=None,
         aux16=None, colsum_part=None, c16_fp16=False, C16b=None):
    """C may be None when only the bf16 copy C16 (same strides) is wanted. Both operands bf16
    (Operand.dtype 1) selects the LDS-DMA kernel (gemm16.hip)."""
    if _state.prec == 3 and A.dtype == 0 and B.dtype == 0 and _x3_single(A, B):
        # bf16x3 policy with a single-pass role (forward on fp16, see _x3_single): this GEMM as in bf16 mode
        kw = dict(locals())
        old = _state.prec
        _state.prec = 0
        try:
            return gemm(**kw)
        finally:
            _state.prec = old
    d = GemmDesc()
    d.M, d.N, d.K = M, N, K
    d.nz1, d.nz2 = nz1, nz2
    d.A = A
    d.B = B
    e = Epilogue()
    e.C = _p(C, c_off)
    e.C16 = _p(C16, c_off)
    e.ldc, e.cbs1, e.cbs2 = ldc, cbs1, cbs2
    e.alpha, e.beta = alpha, beta
    e.bias = _p(bias)
    e.biasbs1 = biasbs1
    e.bias_gather = None if bias_gather is None else bias_gather.data_ptr()
    e.pre_out = _p(pre_out, c_off) if pre_out is not None else None
    e.act, e.act_bwd = act, act_bwd
    e.aux = _p(aux, c_off) if aux is not None else None
    e.ldaux, e.abs1, e.abs2 = ldaux or ldc, abs1 or cbs1, abs2 or cbs2
    e.drop_p = drop_p
    e.drop_seed = seed
    e.residual = _p(residual, r_off) if residual is not None else None
    e.ldr, e.rbs1, e.rbs2 = ldr or ldc, rbs1 or cbs1, rbs2 or cbs2
    e.pre16 = _p(pre16, c_off) if pre16 is not None else None
    e.aux16 = _p(aux16, c_off) if aux16 is not None else None
    e.colsum_part = _p(colsum_part)
    e.C16b = _p(C16b, c_off) if C16b is not None else None
    e.flags = _lib.EPI_C16_FP16 if c16_fp16 else 0
    d.ep = e
    d.precision = 2 if ((_state.fwd16 and _state.prec == 0 and A.dtype == 0) or A.dtype == 2) else _prec()
    keep16 = None
    if _AUTO16 and _state.prec == 0 and A.dtype == 0 and B.dtype == 0 and _auto16_ok(M, N, K, A, B, nz1, nz2):
        # fp32 operands of a large plain GEMM: stage 16-bit copies (the rounding the fp32-operand
        # kernel applies while loading LDS) and run the LDS-DMA kernel (gemm16.hip) on them
        h = d.precision == 2
        dev = (C if C is not None else C16).device
        keep16 = (_cast_operand(A, M, K, h, dev), _cast_operand(B, N, K, h, dev))
        A, B = keep16[0][1], keep16[1][1]
        d.A, d.B = A, B
    d.flops = 2.0 * M * N * K * nz1 * nz2   # algorithmic (the bf16x3 image below triples the MFMA work)
    if _X3_SPLIT[0] and _state.prec == 3 and A.dtype == 0 and B.dtype == 0 and _auto16_ok(M, N, K, A, B, nz1, nz2):
        # bf16x3: split-bf16 images of both operands over K' = 3K, one launch on the bf16 LDS-DMA kernels
        dev = (C if C is not None else C16).device
        form = _x3_form(A, B)
        if form in ("2a", "2b"):   # two-term images over K' = 2K: (hi, lo) . (hi, hi) or the reverse
            pa, pb = (0b10, 0b00) if form == "2a" else (0b00, 0b10)
            keep16 = (_split3_operand(A, M, K, pa | _SPLIT2, dev), _split3_operand(B, N, K, pb | _SPLIT2, dev))
        else:
            keep16 = (_split3_operand(A, M, K, 0b010, dev), _split3_operand(B, N, K, 0b100, dev))
        A, B = keep16[0][1], keep16[1][1]
        d.A, d.B = A, B
        K = (2 if form in ("2a", "2b") else 3) * K
        d.K = K
        d.precision = 0
    d.timing_family = timing or _GEMM_TIMING[0]
    ws = None
    plain = (bias is None and pre_out is None and act == 0 and act_bwd == 0 and drop_p == 0.0 and residual is None
             and colsum_part is None and pre16 is None and C16b is None)
    if plain and K >= 2048 and not _state.nosplit:
        b16 = A.dtype != 0
        bn = 64 if (N <= 64 and not b16) else 128
        blocks = -(-M // 128) * -(-N // bn) * nz1 * nz2
        ks = 1
        tpp = -(-M // 256) * -(-N // 256) * nz1 * nz2
        kpp = min(-(-160 // tpp), K // 1024)
        if (b16 and (_PP_SPLIT or M * N * nz1 * nz2 >= _PP_MIN_MN) and tpp * kpp >= 160 and kpp >= 2
                and (blocks < _PP_SPLIT_MAX_BLOCKS or K >= _PP_SPLIT_LONG_K)):
            # 256x256 ping-pong tiles (gemm16.hip) over >= 1024-deep K slices, ~160-200 workgroups
            # (the frozen weight gradients, K = tokens): fewer, larger tiles than the 128 x 128 split
            ks = kpp
        elif blocks < 240:
            ks = min(-(-_SPLITK_WGS // blocks), K // 1024)
        if ks >= 2:
            q = 64 if b16 else 32
            kchunk = -(-K // ks)
            kchunk = -(-kchunk // q) * q
            ks = -(-K // kchunk)
            dev = (C if C is not None else C16).device
            # slabs + one arrival counter per 128 x 128 output tile (the 16-bit kernel's in-kernel fix-up)
            ctr = -(-M // 128) * -(-N // 128) * nz1 * nz2 if _SPLITK_CTR[0] else 0
            ws = torch.empty(ks * nz1 * nz2 * M * N + ctr, device=dev, dtype=torch.float32)
            d.ksplit, d.kchunk = ks, kchunk
            d.workspace = ws.data_ptr()
            d.workspace_floats = ws.numel()
    if GEMM_LOG is not None:
        GEMM_LOG.append(dict(M=M, N=N, K=K, nz=nz1 * nz2, a16=int(A.dtype), ak=int(A.inner_is_k), bk=int(B.inner_is_k),
                             aconv=int(A.conv), bconv=int(B.conv), ksplit=int(d.ksplit),
                             epi="".join(c for c, f in (("b", bias is not None), ("a", act != 0), ("g", act_bwd != 0),
                                                        ("d", drop_p > 0), ("r", residual is not None),
                                                        ("h", C16 is not None), ("B", C16b is not None),
                                                        ("f", C is not None)) if f),
                             # output-side bytes the epilogue must move once (writes + residual / aux / C reads)
                             out_bytes=M * N * nz1 * nz2 * (4 * (C is not None) + 4 * (pre_out is not None)
                                                            + 2 * (C16 is not None) + 2 * (pre16 is not None)
                                                            + 2 * (C16b is not None)
                                                            + 4 * (residual is not None) + 4 * (beta != 0.0)
                                                            + (2 if aux16 is not None else 4 if aux is not None else 0))))
    _lib.check(_lib.load().b2p_gemm(ctypes.byref(d), _st()), "b2p_gemm")


def _x3_role(A, B) -> str:
    """The role of a bf16x3-mode fp32-operand GEMM by the operand layouts of a Linear: forward (inside
    forward_f16), backward-data (A k-contiguous, B n-contiguous) or weight gradient (both m/n-contiguous)."""
    if _state.fwd16:
        return "fwd"
    if A.inner_is_k and not B.inner_is_k:
        return "dgrad"
    if not A.inner_is_k and not B.inner_is_k:
        return "wgrad"
    return "other"


def _x3_form(A, B) -> str:
    """How the bf16x3 mode runs this GEMM (B2P_X3_SINGLE / the Trainer policy's role set, or the
    diagnostic switches of tools/traj_err_ft.py): '' split-bf16 three-term images; '1' single pass as in
    the bf16 mode (forward on fp16 operands); '2a' / '2b' two-term images (hi*hi + lo*hi: A kept to
    ~16 bits, B rounded to bf16 / the reverse)."""
    forms = _state.x3forms if _state.x3forms is not None else _X3_SINGLE
    if not forms and not DIAG_SWITCHES:
        return ""
    role = _x3_role(A, B)
    for form in ("1", "2a", "2b"):
        if role + form in forms or role + form in DIAG_SWITCHES or (form == "1" and role in forms):
            return form
    return ""


def _x3_single(A, B) -> bool:
    return _x3_form(A, B) == "1"


_X3_SINGLE = set(filter(None, os.environ.get("B2P_X3_SINGLE", "").split(",")))

# The Trainer's bf16x3 policy (configs[4]: the w2v encoder trained) runs the weight-gradient GEMMs
# single-pass (bf16) and the backward-data GEMMs on two-term images (the gradient rounded to bf16, the
# weight kept to ~16 bits); forward GEMMs stay three-term. Measured on conformer_large_ft_bs8 against the
# reference's trajectory (tools/ft_policy_ab.py, profiles/r06m_ft_policy_ab.txt): three-term everywhere
# 8.1e-5 at step 3, 91.6 ms/step; this set 2.1e-4, 83.6 ms; forward single-pass (fp16) or two-term
# 3.1e-3 .. 1.4e-2, backward-data single-pass 2.2e-3 (both past the 1e-3 gate).
# B2P_X3_POLICY=<roles> overrides it ('none': three-term everywhere).
X3_POLICY_FORMS = frozenset(filter(None, os.environ.get("B2P_X3_POLICY", "wgrad,dgrad2b").replace("none", "").split(",")))


def x3_mfma_work(forms) -> float:
    """bf16 MFMA products per algorithmic multiply-add of a bf16x3 step under `forms`, the three GEMM
    roles (forward, backward-data, weight gradient) weighted equally (each ~1/3 of a Linear's FLOPs)."""
    def terms(role):
        for form, n in (("1", 1), ("2a", 2), ("2b", 2)):
            if role + form in forms or (form == "1" and role in forms):
                return n
        return 3
    return sum(terms(r) for r in ("fwd", "dgrad", "wgrad")) / 3.0


@contextlib.contextmanager
def x3_forms(forms):
    """The bf16x3 mode's per-role GEMM forms inside (see _x3_form; None: B2P_X3_SINGLE)."""
    old = _state.x3forms
    _state.x3forms = None if forms is None else frozenset(forms)
    try:
        yield
    finally:
        _state.x3forms = old


# bf16x3 mode: large plain fp32-operand GEMMs run as one bf16 GEMM over split-bf16 operand images
# (B2P_X3_SPLIT=0: the fp32-operand kernel's three-MFMA form, csrc/gemm.hip precision 3)
_X3_SPLIT = [os.environ.get("B2P_X3_SPLIT", "1") != "0"]


_SPLIT2 = 0x10   # b2p_split3_bf16 pattern flag: two K-blocks instead of three


def _split3_operand(o, mn, K, pattern, dev):
    """The split-bf16 image of the logical (mn x K) fp32 operand o: three (pattern & _SPLIT2: two)
    K-blocks (hi / lo per pattern bit), along the rows of a k-contiguous operand, stacked for an
    m/n-contiguous one; (buffer, Operand)."""
    rows, cols = (mn, K) if o.inner_is_k else (K, mn)
    along = bool(o.inner_is_k)
    nb = 2 if pattern & _SPLIT2 else 3
    ld16 = -(-(nb * cols if along else cols) // 8) * 8
    buf = torch.empty(rows if along else nb * rows, ld16, device=dev, dtype=BF16)
    _lib.call("b2p_split3_bf16", o.ptr, rows, cols, o.ld, buf.data_ptr(), ld16, pattern, int(along), _st())
    n = Operand()
    n.ptr = buf.data_ptr()
    n.ld = ld16
    n.bs1 = n.bs2 = 0
    n.gather1 = None
    n.inner_is_k = o.inner_is_k
    n.conv = 0
    n.dtype = 1
    return buf, n


# split-K fix-up inside the 16-bit GEMM (counters behind the slabs); False: the separate reduce launch
_SPLITK_CTR = [True]

# tools/gemm_census.py: when a list, every gemm() call appends its shape record
GEMM_LOG = None

# fp32-operand GEMMs at least this large (2*M*N*K) are run on staged 16-bit operand copies
_AUTO16 = os.environ.get("B2P_GEMM_AUTO16", "1") == "1"
_AUTO16_MIN_FLOP = float(os.environ.get("B2P_GEMM_AUTO16_MIN_GFLOP", "2")) * 1e9


def _auto16_ok(M, N, K, A, B, nz1, nz2) -> bool:
    """Plain single-matrix operands (no implicit conv view, gather or batch) in a layout the 16-bit
    kernel takes, and enough work to amortise the two cast passes."""
    if nz1 * nz2 != 1 or A.conv or B.conv or A.gather1 or B.gather1:
        return False
    if not A.inner_is_k and B.inner_is_k:
        return False
    if (A.inner_is_k or B.inner_is_k) and K % 8 != 0:
        return False
    return 2.0 * M * N * K >= _AUTO16_MIN_FLOP and min(M, N) >= 64 and K >= 64


_FROZEN_PTR: dict = {}   # data_ptr -> frozen parameter (set_deferred_wgrad)
_FROZEN_ROLE: dict = {}  # id -> the frozen parameter's name with layer indices masked (set_deferred_wgrad)
_CAST_CACHE: dict = {}   # (ptr, rows, cols, ld, fp16) -> (version, buffer) for frozen parameters


def _cast_operand(o, mn, K, fp16, dev):
    """16-bit compact copy of the logical (mn x K) operand o (row stride rounded up to 8 elements);
    returns (buffer, Operand). Copies of frozen parameters are cached across calls."""
    rows, cols = (mn, K) if o.inner_is_k else (K, mn)
    ld16 = -(-cols // 8) * 8
    prm = _FROZEN_PTR.get(o.ptr)
    key = (o.ptr, rows, cols, o.ld, bool(fp16))
    buf = None
    if prm is not None and prm.numel() >= rows * o.ld - (o.ld - cols):
        hit = _CAST_CACHE.get(key)
        if hit is not None and hit[0] == prm._version:
            buf = hit[1]
    else:
        prm = None
    if buf is None:
        buf = torch.empty(rows, ld16, device=dev, dtype=torch.float16 if fp16 else BF16)
        _lib.call("b2p_cast16_2d", o.ptr, rows, cols, o.ld, buf.data_ptr(), ld16, int(fp16), _st())
        if prm is not None:
            _CAST_CACHE[key] = (prm._version, buf)
    n = Operand()
    n.ptr = buf.data_ptr()
    n.ld = ld16
    n.bs1 = n.bs2 = 0
    n.gather1 = None
    n.inner_is_k = o.inner_is_k
    n.conv = 0
    n.dtype = 2 if fp16 else 1
    return buf, n


def mm_nt(x, W, out, bias=None, act=0, pre_out=None, drop_p=0.0, seed=0, residual=None, alpha=1.0, beta=0.0,
          timing=0):
    """out[M,N] = epi(x[M,K] @ W[N,K]^T) (nn.Linear forward)."""
    M, K = x.shape[-2] if x.dim() > 1 else 1, x.shape[-1]
    M = x.numel() // K
    N = W.shape[0]
    gemm(M, N, K, op(x, 0, K, True), op(W, 0, W.shape[1], True), out, N, bias=bias, act=act, pre_out=pre_out,
         drop_p=drop_p, seed=seed, residual=residual, alpha=alpha, beta=beta, timing=timing)


def mm_nn(a, W, out, act_bwd=0, aux=None, drop_p=0.0, seed=0, residual=None, alpha=1.0, beta=0.0):
    """out[M,N] = epi(a[M,K] @ W[K,N]) (nn.Linear input gradient, W = weight [out,in])."""
    K, N = W.shape[0], W.shape[1]
    M = a.numel() // K
    gemm(M, N, K, op(a, 0, K, True), op(W, 0, N, False), out, N, act_bwd=act_bwd, aux=aux, drop_p=drop_p,
         seed=seed, residual=residual, alpha=alpha, beta=beta)


def mm_tn(dy, x, out, beta=0.0):
    """out[N,K] = dy[M,N]^T @ x[M,K] (nn.Linear weight gradient)."""
    N = dy.shape[-1]
    K = x.shape[-1]
    M = dy.numel() // N
    gemm(N, K, M, op(dy, 0, N, False), op(x, 0, K, False), out, K, beta=beta)


_WS = {}


def _colsum_ws(M, N, device):
    n = int(_lib.load().b2p_colsum_workspace(M, N))
    return torch.empty(max(n, 1), device=device, dtype=torch.float32)


def colsum_parts_buf(M, N, device):
    """Workspace for a GEMM epilogue's fused column sums (one partial row per 32 output rows: every wave row
    block of the GEMM kernels, 64 / 96 / 128 rows, starts on a 32-row band)."""
    return torch.empty(-(-M // 32), N, device=device)


def colsum_from_parts(parts, out):
    _lib.call("b2p_colsum_parts", _p(parts), parts.shape[0], parts.shape[1], _p(out), 0, _st())
    return out


class ColsumParts:
    """Column sums still held as per-tile partial rows (a GEMM epilogue's colsum_part or
    b2p_drop_cast_colsum's): a frozen parameter's deferred accumulation finishes them inside the
    side stream's batched launch (b2p_accum_rows_recs), everything else calls materialize()."""
    __slots__ = ("parts",)

    def __init__(self, parts):
        self.parts = parts

    def materialize(self):
        return colsum_from_parts(self.parts, torch.empty(self.parts.shape[1], device=self.parts.device))


def _mat(g):
    return g.materialize() if isinstance(g, ColsumParts) else g


# B2P_LAZY_COLSUM=0 (A/B): deferred bias gradients are finished by a colsum_p2 launch on the main
# stream, as before, instead of inside the side stream's batched accumulation
_LAZY_COLSUM = os.environ.get("B2P_LAZY_COLSUM", "1") != "0"


def colsum(x2d_ptr_tensor, M, N, out, ld=None, accumulate=False):
    ws = _colsum_ws(M, N, out.device)
    _lib.call("b2p_colsum", _p(x2d_ptr_tensor), M, N, ld or N, _p(out), int(accumulate), _p(ws), _st())


def colsum_batched(x, batch, M, N, out, ld=None, bstride=None, mode=0, y=None):
    ws = torch.empty(max(int(_lib.load().b2p_colsum_workspace(M, N)) * batch, 1), device=out.device)
    _lib.call("b2p_colsum_batched", _p(x), _p(y), batch, M, N, ld or N, bstride if bstride is not None else M * N,
              mode, _p(out), 0, _p(ws), _st())


def _dropout_raw(x, p, seed, out=None):
    out = torch.empty_like(x) if out is None else out
    _lib.call("b2p_dropout", _p(x), _p(out), x.numel(), float(p), seed, _st())
    return out


def _act_bwd(dy, pre, act, out=None):
    out = torch.empty_like(dy) if out is None else out
    _lib.call("b2p_act_bwd", _p(dy), _p(pre), _p(out), dy.numel(), act, _st())
    return out


def _ln_fwd(x2d, g, b, eps, drop_p=0.0, seed=0):
    rows, cols = x2d.shape
    y = torch.empty_like(x2d)
    mean = torch.empty(rows, device=x2d.device)
    rstd = torch.empty(rows, device=x2d.device)
    _lib.call("b2p_layernorm_fwd", _p(x2d), _p(g), _p(b), _p(y), _p(mean), _p(rstd), rows, cols, float(eps),
              float(drop_p), seed, _st())
    return y, mean, rstd


_LN_BWD_ROWS = 16   # rows per block of ln_bwd_k (csrc/elementwise.hip LN_BWD_ROWS): the partials' row count
_LN_LAZY = os.environ.get("B2P_LN_LAZY", "1") != "0"   # B2P_LN_LAZY=0: reduce them on the main stream (A/B)


def _ln_lazy(lazy, need_params, dbias_in) -> bool:
    """The LayerNorm backward leaves its parameter gradients as block partials (ColsumParts, finished in
    the side stream's batched accumulation) when every parameter they belong to is a deferred frozen
    one: lazy = (gamma, beta, the dropout-input bias or None), matching dbias_in."""
    return (_LAZY_COLSUM and _LN_LAZY and lazy is not None and need_params and (dbias_in is None) == (lazy[2] is None)
            and all(_defer_ok(q) for q in lazy if q is not None))


def _ln_parts(ws, rows, cols, q):
    nblk = -(-rows // _LN_BWD_ROWS)
    return ColsumParts(ws[q * nblk * cols:(q + 1) * nblk * cols].view(nblk, cols))


def _ln_bwd(dy, x, g, mean, rstd, need_params=True, dx_accum=None, drop_p=0.0, seed=0, in_drop_p=-1.0,
            in_seed=0, dbias_in=None, dx_accum2=None, lazy=None):
    """dx_accum2: a second accumulator added to dx alone (LayerDrop's skip gradient, _skip_take).
    lazy (see _ln_lazy): dg / db come back as ColsumParts (no ln_param_reduce launch on the main stream),
    and the result gains a fifth entry, the dropout-input bias gradient (dbias_in or its ColsumParts)."""
    rows, cols = x.shape
    lz = _ln_lazy(lazy, need_params, dbias_in)
    dx = torch.empty_like(x)
    dg = torch.empty(cols, device=x.device) if need_params and not lz else None
    db = torch.empty(cols, device=x.device) if need_params and not lz else None
    ws = torch.empty(int(_lib.load().b2p_layernorm_bwd_workspace(rows, cols)), device=x.device)
    dxd = torch.empty_like(x) if in_drop_p >= 0.0 else None
    _lib.call("b2p_layernorm_bwd_acc2", _p(dy), _p(x), _p(g), _p(mean), _p(rstd), _p(dx), _p(dg), _p(db), rows,
              cols, _p(dx_accum), _p(dx_accum2), float(drop_p), seed, _p(dxd), float(max(in_drop_p, 0.0)), in_seed,
              None if lz else _p(dbias_in), None, _p(ws), _st())
    if lz:
        dg, db = _ln_parts(ws, rows, cols, 0), _ln_parts(ws, rows, cols, 1)
        dbias_in = _ln_parts(ws, rows, cols, 2) if dbias_in is not None else None
    return (dx, dg, db, dxd) if lazy is None else (dx, dg, db, dxd, dbias_in)



# ------------------------------------------------------------------ bf16 GEMM operands
# In bf16 mode every large GEMM reads bf16 copies of its operands straight into LDS (gemm16.hip).
# Master weights, activations needed by elementwise kernels, and all gradients stay fp32; the
# bf16 copies are written by the producing kernel (GEMM epilogue C16, LayerNorm y16/d16) or by
# one cast. Rounding is the same RNE fp32->bf16 the fp32-operand kernel applies while staging,
# so both paths compute the same products.
BF16 = torch.bfloat16
_PARAM_EPOCH: dict = {}
_W16: dict = {}


def _bwd16_path() -> bool:
    """A block backward takes its 16-bit-operand form (not under the bwd32path diagnostic)."""
    return bf16_mode() and "bwd32path" not in DIAG_SWITCHES


def bf16_mode() -> bool:
    return _prec() == 0


def bump_param_epoch(params) -> None:
    """Called by optimisers that update parameters in place through raw pointers (HipAdam):
    torch's version counter does not see those writes, so cached bf16 weight copies would go
    stale without this."""
    for p in params:
        _PARAM_EPOCH[id(p)] = _PARAM_EPOCH.get(id(p), 0) + 1


class _Stamp:
    """Identity + content stamp of the source weights of a cached 16-bit copy. Weak references make
    a freed weight a miss even when a new tensor reuses its id, storage and version counter (models
    built one after another in one process)."""
    __slots__ = ("key", "refs")

    def __init__(self, ws):
        self.key = tuple((id(w), w.data_ptr(), tuple(w.shape), w._version, _PARAM_EPOCH.get(id(w), 0)) for w in ws)
        self.refs = tuple(weakref.ref(w) for w in ws)

    def __eq__(self, other):
        return (isinstance(other, _Stamp) and self.key == other.key
                and all(a() is not None and a() is b() for a, b in zip(self.refs, other.refs)))


def _stamp(ws):
    return _Stamp(ws)


def _cache_ok(ws) -> bool:
    """Inside a graph capture only frozen parameters (set_deferred_wgrad) may come from or go to the
    weight-copy cache: the copy of a trained weight must be a node of the graph, so that every replay
    reads the weight the previous replay's (captured or eager) optimizer step wrote."""
    return not capturing() or all(id(w) in _Deferred.ids for w in ws)


def cast16(x, out=None):
    out = torch.empty(x.shape, device=x.device, dtype=BF16) if out is None else out
    _lib.call("b2p_cast_bf16", _p(x), _p(out), x.numel(), _st())
    return out


def weight16(*ws, half=False):
    """bf16 (fp16 when half) copy of fp32 weight(s), rows concatenated ([wq; wk; wv] -> one QKV
    operand); cached until any source tensor changes (version counter or optimiser epoch)."""
    key = (("H",) if half else ()) + tuple(id(w) for w in ws)
    st = _stamp(ws)
    cache = _cache_ok(ws)
    hit = _W16.get(key) if cache else None
    if hit is not None and hit[0] == st:
        return hit[1]
    rows = sum(w.shape[0] for w in ws)
    out = torch.empty((rows,) + tuple(ws[0].shape[1:]), device=ws[0].device, dtype=torch.float16 if half else BF16)
    off = 0
    for w in ws:
        _chk(w, "weight16")
        if half:
            _lib.call("b2p_cast16_2d", _p(w), 1, w.numel(), w.numel(), _p(out, off), w.numel(), 1, _st())
        else:
            _lib.call("b2p_cast_bf16", _p(w), _p(out, off), w.numel(), _st())
        off += w.numel()
    if cache:
        _W16[key] = (st, out)
    return out


_BS: dict = {}


def _scaled_bias(b, scale):
    """b * scale (the macaron FFN's half-step output bias, TF conf EncoderLayer: x + 0.5 * ffn(x)), cached
    like the 16-bit weight copies: a frozen bias costs no launch per step."""
    if b is None:
        return None
    key = (id(b), float(scale))
    st = _stamp((b,))
    cache = _cache_ok((b,))
    hit = _BS.get(key) if cache else None
    if hit is not None and hit[0] == st:
        return hit[1]
    out = b * scale
    if cache:
        _BS[key] = (st, out)
    return out


def weight16t(*ws):
    """Transposed bf16 copy [C][sum R] of fp32 weights (R x C each, stacked along R): the
    k-contiguous B operand of a backward-data GEMM dX = dY W (NT kernel instead of the slower
    transposed-read NN form); cached like weight16."""
    key = ("T",) + tuple(id(w) for w in ws)
    st = _stamp(ws)
    cache = _cache_ok(ws)
    hit = _W16.get(key) if cache else None
    if hit is not None and hit[0] == st:
        return hit[1]
    rows = sum(w.shape[0] for w in ws)
    C = ws[0].shape[1]
    out = torch.empty(C, rows, device=ws[0].device, dtype=BF16)
    off = 0
    for w in ws:
        _chk(w, "weight16t")
        _lib.call("b2p_transpose_bf16", _p(w), _p(out), w.shape[0], C, rows, off, _st())
        off += w.shape[0]
    if cache:
        _W16[key] = (st, out)
    return out


def bias_cat(*bs):
    """fp32 concatenation of biases (None -> zeros), cached like weight16."""
    ref = next(b for b in bs if b is not None)
    real = tuple(b for b in bs if b is not None)
    key = ("bias",) + tuple(id(b) if b is not None else None for b in bs)
    st = _stamp(real)
    cache = _cache_ok(real)
    hit = _W16.get(key) if cache else None
    if hit is not None and hit[0] == st:
        return hit[1]
    out = torch.zeros(sum(ref.numel() for _ in bs), device=ref.device)
    n = ref.numel()
    for i, b in enumerate(bs):
        if b is not None:
            out[i * n:(i + 1) * n].copy_(b)
    if cache:
        _W16[key] = (st, out)
    return out


def attach16(x, x16) -> None:
    """Marks x16 as the bf16 copy of x (consumed by the next op's GEMM instead of a cast)."""
    x._b16 = (x._version, x16)


def to16(x):
    t = getattr(x, "_b16", None)
    if t is not None and t[0] == x._version:
        return t[1]
    return cast16(x.contiguous())


def attach16h(x, xh) -> None:
    """Marks xh as the fp16 copy of x (the forward_f16 GEMM operand), beside attach16's bf16 copy."""
    x._h16 = (x._version, xh)


def to16h(x):
    t = getattr(x, "_h16", None)
    if t is not None and t[0] == x._version:
        return t[1]
    xc = x.contiguous()
    out = torch.empty(xc.shape, device=x.device, dtype=torch.float16)
    _lib.call("b2p_cast16_2d", _p(xc), 1, xc.numel(), xc.numel(), _p(out), xc.numel(), 1, _st())
    return out


def _ln_fwd16(x2d, g, b, eps, drop_p=0.0, seed=0):
    rows, cols = x2d.shape
    y = torch.empty_like(x2d)
    y16 = torch.empty(rows, cols, device=x2d.device, dtype=BF16)
    mean = torch.empty(rows, device=x2d.device)
    rstd = torch.empty(rows, device=x2d.device)
    _lib.call("b2p_layernorm_fwd16", _p(x2d), _p(g), _p(b), _p(y), _p(y16), _p(mean), _p(rstd), rows, cols,
              float(eps), float(drop_p), seed, _st())
    return y, y16, mean, rstd


def _ln_bwd16(dy, x, g, mean, rstd, need_params=True, dx_accum=None, drop_p=0.0, seed=0, in_drop_p=-1.0,
              in_seed=0, dbias_in=None, dx_accum2=None, lazy=None):
    """as _ln_bwd, plus d16 = bf16(dx_dropped if in_drop_p >= 0 else dx) (lazy: a sixth entry, the
    dropout-input bias gradient)"""
    rows, cols = x.shape
    lz = _ln_lazy(lazy, need_params, dbias_in)
    dx = torch.empty_like(x)
    dg = torch.empty(cols, device=x.device) if need_params and not lz else None
    db = torch.empty(cols, device=x.device) if need_params and not lz else None
    ws = torch.empty(int(_lib.load().b2p_layernorm_bwd_workspace(rows, cols)), device=x.device)
    dxd = torch.empty_like(x) if in_drop_p >= 0.0 else None
    d16 = torch.empty(rows, cols, device=x.device, dtype=BF16)
    _lib.call("b2p_layernorm_bwd_acc2", _p(dy), _p(x), _p(g), _p(mean), _p(rstd), _p(dx), _p(dg), _p(db), rows,
              cols, _p(dx_accum), _p(dx_accum2), float(drop_p), seed, _p(dxd), float(max(in_drop_p, 0.0)), in_seed,
              None if lz else _p(dbias_in), _p(d16), _p(ws), _st())
    if lz:
        dg, db = _ln_parts(ws, rows, cols, 0), _ln_parts(ws, rows, cols, 1)
        dbias_in = _ln_parts(ws, rows, cols, 2) if dbias_in is not None else None
    return (dx, dg, db, dxd, d16) if lazy is None else (dx, dg, db, dxd, d16, dbias_in)


# =====================================================================================
# front end: GaussianSmoothing -> day linear (+bias) -> softsign
# =====================================================================================
@_prec_follow
class _FrontEnd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, day_idxs, day_weights, day_bias, taps):
        _chk(x, "front_end.x")
        _chk(day_weights, "front_end.day_weights")
        B, L, C = x.shape
        xs = torch.empty_like(x)
        _lib.call("b2p_gauss_smooth", _p(x), _p(taps), taps.numel(), _p(xs), B, L, C, _st())
        z = torch.empty_like(x)
        s = torch.empty_like(x)
        # z[b] = xs[b] @ W[day[b]] + bias[day[b]] ; s = softsign(z)   (einsum "btd,bdk->btk")
        gemm(L, C, C, op(xs, 0, C, True, bs1=L * C), op(day_weights, 0, C, False, bs1=C * C, gather=day_idxs),
             s, C, cbs1=L * C, nz1=B, bias=day_bias, biasbs1=C, bias_gather=day_idxs, pre_out=z,
             act=ACT["softsign"])
        ctx.save_for_backward(xs, z, day_idxs, day_weights)
        ctx.n_days = day_weights.shape[0]
        return s

    @staticmethod
    def backward(ctx, ds):
        xs, z, day_idxs, day_weights = ctx.saved_tensors
        ds = ds.contiguous()
        B, L, C = xs.shape
        dz = _act_bwd(ds, z, ACT["softsign"])
        dW = dbias = None
        if ctx.needs_input_grad[2]:
            per = torch.empty(B, C, C, device=xs.device)
            # per[b] = xs[b]^T @ dz[b]   (K = L), then summed per day (deterministic)
            gemm(C, C, L, op(xs, 0, C, False, bs1=L * C), op(dz, 0, C, False, bs1=L * C), per, C, cbs1=C * C, nz1=B)
            dW = torch.empty_like(day_weights)
            _lib.call("b2p_day_reduce", _p(per), _p(day_idxs), B, ctx.n_days, C * C, _p(dW), _st())
        if ctx.needs_input_grad[3]:
            per_b = torch.empty(B, C, device=xs.device)
            colsum_batched(dz, B, L, C, per_b)
            dbias = torch.empty(ctx.n_days, 1, C, device=xs.device)
            _lib.call("b2p_day_reduce", _p(per_b), _p(day_idxs), B, ctx.n_days, C, _p(dbias), _st())
        return None, None, dW, dbias, None


def front_end(x, day_idxs, day_weights, day_bias, taps):
    """b2p2t_model.py:150-159: permute -> GaussianSmoothing -> einsum(btd,bdk) + day_bias -> Softsign.
    Returns the (B, L, 256) softsign output (the Unfold is implicit in the GRU layer-0 projection)."""
    with _fp32_if("front"):
        return _FrontEnd.apply(x.contiguous(), day_idxs.to(torch.int64).contiguous(), day_weights, day_bias, taps)


# =====================================================================================
# GRU layer (both directions)
# =====================================================================================
class Unfolded:
    """Lazy nn.Unfold((k,1), stride) view of a (B, L, C) tensor (b2p2t_model.py:108-113, 162-167):
    logically (B, T, C*k) with T = (L-k)//stride + 1. Never materialised on the product path; the
    GRU layer-0 projection reads it as an implicit-GEMM operand."""

    def __init__(self, src: torch.Tensor, kernel: int, stride: int):
        self.src = src
        self.kernel = kernel
        self.stride = stride
        B, L, C = src.shape
        self.T = (L - kernel) // stride + 1
        self.shape = (B, self.T, C * kernel)

    def materialize(self) -> torch.Tensor:
        """Reference layout (feature index c*k + tap); for inspection/tests only."""
        B, L, C = self.src.shape
        idx = torch.arange(self.T, device=self.src.device)[:, None] * self.stride + torch.arange(self.kernel, device=self.src.device)[None, :]
        win = self.src[:, idx, :]                      # (B, T, k, C)
        return win.permute(0, 1, 3, 2).reshape(B, self.T, C * self.kernel)


# bf16 mode's GRU layer 0 reads the Unfold through an implicit overlapping-row view (B2P_UNFOLD_IMPLICIT=0:
# the materialised bf16 unfold + col2im of round 3, for A/B checks)
_UNFOLD_IMPLICIT = [os.environ.get("B2P_UNFOLD_IMPLICIT", "1") != "0"]
# persistent MFMA recurrence in bf16 mode (B2P_GRU16=0 selects the per-step fp32 kernels, for A/B checks)
_GRU16 = [os.environ.get("B2P_GRU16", "1") != "0"]
# hidden sizes one CU cannot hold (Conformer H = 512): the multi-CU persistent kernels (csrc/grumc.hip)
# in bf16 mode (B2P_GRUMC=0: per-step kernels, for A/B checks)
_GRUMC = [os.environ.get("B2P_GRUMC", "1") != "0"]
# diagnostic (tools/traj_err.py): None = the backward follows the forward's choice; True / False force
# the multi-CU / per-step fp32 backward recurrence (same saved layout)
_GRUMC_BWD = [None]


def _gru_mc_ws(B, H, ndir, dev):
    return torch.empty(int(_lib.load().b2p_gru_mc_workspace(B, H, ndir)), device=dev, dtype=torch.uint8)


# Multi-CU GRU timeouts (csrc/grumc.hip): a member that never publishes its state leaves the others
# to time out with garbage results. Every launch folds its timeout flag into one persistent device
# word per device (b2p_gru_mc_status: the first failure's code is kept); the host reads it at its
# next sync (the loss readback of a forward with sync_metrics, the Trainer after a replay) and raises.
_GRU_STATUS: dict = {}      # device -> int32[1]
_GRU_LAYERS: dict = {}      # id(W_hh of direction 0) -> layer number (order of first use)


def _gru_status_word(dev):
    st = _GRU_STATUS.get(dev)
    if st is None:
        st = _GRU_STATUS[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return st


def _gru_mc_code(kind: int, whh0, H: int) -> int:
    n = _GRU_LAYERS.setdefault(id(whh0), len(_GRU_LAYERS))
    return kind * 65536 + (n % 4096) * 16 + {256: 1, 384: 2, 512: 3}.get(H, 0)


def _gru_mc_fold(ws, kind, whh0, H, dev):
    _lib.call("b2p_gru_mc_status", _p(ws), _p(_gru_status_word(dev)), _gru_mc_code(kind, whh0, H), _st())


def _gru_status_error(code: int) -> RuntimeError:
    kind = {1: "forward", 2: "backward"}.get(code // 65536, "?")
    n, h = (code % 65536) // 16, {1: 256, 2: 384, 3: 512}.get(code % 16, "?")
    return RuntimeError(f"multi-CU GRU recurrence timed out ({kind} of GRU layer {n}, H={h}; recurrence id "
                        f"{code}): a member workgroup never published its state (not co-resident?), so the "
                        "layer's outputs / gradients of that step are invalid")


def gru_status_value(dev=None) -> int:
    """Current status word (0 = no multi-CU GRU timeout since the last check); a host sync."""
    dev = dev if dev is not None else torch.device("cuda", torch.cuda.current_device())
    st = _GRU_STATUS.get(torch.device(dev))
    return 0 if st is None else int(st.item())


def check_gru_status(dev=None) -> None:
    """Raises RuntimeError if a multi-CU GRU launch on `dev` (default: every device used) timed out
    since the last check (then the word is cleared). One host sync per device."""
    for d, st in list(_GRU_STATUS.items()):
        if dev is not None and d != torch.device(dev):
            continue
        code = int(st.item())
        if code:
            st.zero_()
            raise _gru_status_error(code)


def loss_item(loss: torch.Tensor) -> float:
    """loss.item() (the reference's per-step readback, w2v_custom_feat_extractor.py:94) with the
    multi-CU GRU status word of the loss's device in the same transfer: raises on a timeout."""
    st = _GRU_STATUS.get(loss.device)
    if st is None:
        return loss.item()
    v, code = torch.stack([loss.detach().reshape(()).float(), st.reshape(()).float()]).tolist()
    if code:
        st.zero_()
        raise _gru_status_error(int(code))
    return v


def _ln_floats(B, T, H, ndir, R):
    return int(_lib.load().b2p_gru16_lane_floats(B, T, H, ndir, R))


def _stack2(a, b):
    return a.unsqueeze(0) if b is None else torch.stack([a, b], 0)


@_prec_follow
class _GRULayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, unf_meta, H, ndir, h0, *weights):
        # weights: per direction (w_ih, w_hh, b_ih, b_hh)  (b_* may be None)
        dev = x.device
        if unf_meta is not None:
            ktaps, stride = unf_meta
            B, L, C = x.shape
            T = (L - ktaps) // stride + 1
            IN = C * ktaps
        else:
            B, T, IN = x.shape
        G3 = 3 * H
        wih = [weights[4 * d + 0] for d in range(ndir)]
        whh = [weights[4 * d + 1] for d in range(ndir)]
        bih = [weights[4 * d + 2] for d in range(ndir)]
        bhh = [weights[4 * d + 3] for d in range(ndir)]
        for w in wih + whh:
            _chk(w, "gru.weight")
        gi = torch.empty(B, T, ndir * G3, device=dev)
        # bf16 mode: persistent MFMA recurrence (csrc/gru16.hip), which wants b_hh's r/z parts folded
        # into the input projection bias
        # the bf16x3 mode's 'grurec1' form (X3_POLICY_FORMS): the persistent recurrences (fp16 / bf16 MFMA on
        # W_hh h) with the input-projection and weight-gradient GEMMs kept in the mode's split-bf16 form
        fast = bf16_mode() or (_state.prec == 3 and "grurec1" in (_state.x3forms if _state.x3forms is not None
                                                                     else _X3_SINGLE))
        use16 = fast and _GRU16[0] and bool(_lib.load().b2p_gru16_supported(H))
        usemc = fast and not use16 and _GRUMC[0] and bool(_lib.load().b2p_gru_mc_supported(H))
        # the step's stacked recurrent weights / biases and the concatenated input-projection bias (with
        # b_hh's r/z parts folded in for gru16), assembled by ONE launch (b2p_gather_recs)
        whh_s = torch.empty(ndir, G3, H, device=dev)
        bhh_s = torch.empty(ndir, G3, device=dev) if bhh[0] is not None else None
        has_bias = any(b is not None for b in bih) or (use16 and bhh[0] is not None)
        bias_cat = torch.empty(ndir * G3, device=dev) if has_bias else None
        recs = []
        for d in range(ndir):
            recs += [_p(whh_s, d * G3 * H), _p(whh[d]), 0, G3 * H]
            if bhh_s is not None:
                recs += [_p(bhh_s, d * G3), _p(bhh[d]), 0, G3]
            if bias_cat is not None:
                fold = use16 and bhh[0] is not None
                recs += [_p(bias_cat, d * G3), _p(bih[d]) or 0, _p(bhh[d]) if fold else 0, 2 * H,
                         _p(bias_cat, d * G3 + 2 * H), _p(bih[d], 2 * H) or 0, 0, H]
        arr = (ctypes.c_int64 * len(recs))(*recs)
        _lib.call("b2p_gather_recs", arr, len(recs) // 4, _st())
        implicit = (unf_meta is not None and bf16_mode() and L % stride == 0 and ktaps % stride == 0 and C % 4 == 0
                    and _UNFOLD_IMPLICIT[0])
        if implicit:
            # implicit Unfold (csrc/elementwise.hip "implicit Unfold operands"): the GEMM reads a 16-bit copy
            # of x through an overlapping-row view (row stride stride*C); fp16 operands under forward_f16
            half = _state.fwd16
            N3 = ndir * G3
            wf = torch.empty(N3, IN, device=dev, dtype=torch.float16 if half else BF16)
            # the backward-data operand of the same weights, written in the same pass when needed
            wperm = (torch.empty((ktaps // stride) * N3, stride * C, device=dev, dtype=BF16)
                     if ctx.needs_input_grad[0] else None)
            _lib.call("b2p_unfold_weight16", _p(wih[0]), _p(wih[1]) if ndir == 2 else None, G3, C, ktaps, stride,
                      _p(wf), int(half), _p(wperm), _st())
            n_s, tail = B * L * C, (ktaps - stride) * C
            s16 = torch.empty(n_s + tail, device=dev, dtype=torch.float16 if half else BF16)
            _lib.call("b2p_cast16_tail", _p(x), _p(s16), n_s, n_s + tail, int(half), _st())
            gemm(T, N3, IN, op(s16, 0, stride * C, True, bs1=L * C), op(wf, 0, IN, True), gi, N3, cbs1=T * N3, nz1=B,
                 bias=bias_cat)
            del wf
            U16 = None if half else s16    # the bf16 copy doubles as the weight-gradient operand
            del s16
        elif unf_meta is not None:
            # tap-major weight copy: W'[n][tap*C + c] = W[n][c*k + tap] for both directions
            wperm = torch.empty(ndir * G3, IN, device=dev)
            for d in range(ndir):
                _lib.call("b2p_conv_weight_permute", _p(wih[d]), _p(wperm, d * G3 * IN), G3, C, ktaps, 0, _st())
            if bf16_mode() and not _state.fwd16:
                # bf16 operands: the tap-major unfold materialised once in bf16 (it is also the
                # weight-gradient operand) and a bf16 copy of the permuted weight
                U16 = torch.empty(B * T, IN, device=dev, dtype=BF16)
                _lib.call("b2p_unfold16", _p(x), _p(U16), B, L, C, ktaps, stride, _st())
                wperm = cast16(wperm)
                gemm(B * T, ndir * G3, IN, op(U16, 0, IN, True), op(wperm, 0, IN, True), gi, ndir * G3, bias=bias_cat)
            else:   # fp32 mode, or fp16 operands (forward_f16): the fp32-operand kernel rounds while staging
                U16 = None
                A = conv_op(x, 0, C, T, L, stride, 0, C * ktaps, L * C, True)
                A.conv_Cg = C  # inner j = tap*C + c
                gemm(B * T, ndir * G3, IN, A, op(wperm, 0, IN, True), gi, ndir * G3, bias=bias_cat)
        else:
            _chk(x, "gru.x")
            wperm = U16 = None
            if bf16_mode() and IN % 8 == 0:
                # both directions' projections as ONE GEMM over the stacked 16-bit W_ih (fp16 under
                # forward_f16), N = ndir * 3H
                half = _state.fwd16
                w16 = torch.empty(ndir * G3, IN, device=dev, dtype=torch.float16 if half else BF16)
                for d in range(ndir):
                    _lib.call("b2p_cast16_2d", _p(wih[d]), G3, IN, IN, _p(w16, d * G3 * IN), IN, int(half), _st())
                x16 = torch.empty(B * T, IN, device=dev, dtype=w16.dtype)
                _lib.call("b2p_cast16_2d", _p(x), B * T, IN, IN, _p(x16), IN, int(half), _st())
                gemm(B * T, ndir * G3, IN, op(x16, 0, IN, True), op(w16, 0, IN, True), gi, ndir * G3, bias=bias_cat)
                del w16, x16
            else:
                for d in range(ndir):
                    gemm(B * T, G3, IN, op(x, 0, IN, True), op(wih[d], 0, IN, True), gi, ndir * G3, c_off=d * G3,
                         bias=None if bias_cat is None else _view_off(bias_cat, d * G3))
        out = torch.empty(B, T, ndir * H, device=dev)
        saved = None if use16 else torch.empty(B, T, ndir, 4, H, device=dev)
        if h0 is not None:
            _chk(h0, "gru.h0")
        if use16:
            # lane-native per-step layouts (csrc/gru16.hip): gi -> giL, kernel, hL -> out
            giL = torch.empty(_ln_floats(B, T, H, ndir, 3), device=dev)
            _lib.call("b2p_gru_lane_permute", _p(gi), _p(giL), B, T, H, ndir, 3, 3, 0x210, 1, _st())
            del gi
            hL = torch.empty(_ln_floats(B, T, H, ndir, 1), device=dev)
            saved = torch.empty(_ln_floats(B, T, H, ndir, 4), device=dev)
            _lib.call("b2p_gru_fwd16", _p(giL), _p(whh_s), _p(bhh_s), _p(h0), _p(hL), _p(saved), B, T, H, ndir,
                      _st())
            del giL
            _lib.call("b2p_gru_lane_permute", _p(hL), _p(out), B, T, H, ndir, 1, 1, 0x0, 0, _st())
        elif usemc:
            hL = None
            ws = _gru_mc_ws(B, H, ndir, dev)
            _lib.call("b2p_gru_fwd_mc", _p(gi), _p(whh_s), _p(bhh_s), _p(h0), _p(out), _p(saved), _p(ws), B, T, H,
                      ndir, _st())
            _gru_mc_fold(ws, 1, whh[0], H, dev)
        else:
            hL = None
            _lib.call("b2p_gru_fwd", _p(gi), _p(whh_s), _p(bhh_s), _p(h0), _p(out), _p(saved), B, T, H, ndir,
                      _st())
        ctx.save_for_backward(x, out, saved, whh_s, h0, wperm, hL, U16, *wih)
        ctx.meta = (unf_meta, H, ndir, B, T, IN, bih[0] is not None, bhh[0] is not None, use16, usemc)
        ctx.implicit = unf_meta is not None and implicit
        ctx.whh0 = whh[0]
        return out

    @staticmethod
    def backward(ctx, dout):
        x, out, saved, whh_s, h0, wperm, hL, U16, *wih = ctx.saved_tensors
        unf_meta, H, ndir, B, T, IN, has_bih, has_bhh, use16, usemc = ctx.meta
        if not use16 and _GRUMC_BWD[0] is not None:
            usemc = _GRUMC_BWD[0] and bool(_lib.load().b2p_gru_mc_supported(H))
        dev = out.device
        dout = dout.contiguous()
        G3 = 3 * H
        dgi = torch.empty(B, T, ndir * G3, device=dev)
        dgh = torch.empty(B, T, ndir * G3, device=dev)
        dh0 = torch.empty(ndir, B, H, device=dev) if (h0 is not None and ctx.needs_input_grad[4]) else None
        if use16:
            doL = torch.empty(_ln_floats(B, T, H, ndir, 1), device=dev)
            _lib.call("b2p_gru_lane_permute", _p(dout), _p(doL), B, T, H, ndir, 1, 1, 0x0, 1, _st())
            dgL = torch.empty(_ln_floats(B, T, H, ndir, 4), device=dev)
            # frozen-parameter gradient GEMMs fill the chip beside the 4-CU recurrence
            _gru_bwd_launch(lambda: _lib.call("b2p_gru_bwd16", _p(doL), _p(whh_s), _p(hL), _p(saved), _p(h0), _p(dgL),
                                              _p(dh0), B, T, H, ndir, _st()))
            del doL
            # dgi = LN records (0, 1, 2), dgh = LN records (0, 1, 3)
            _lib.call("b2p_gru_lane_permute", _p(dgL), _p(dgi), B, T, H, ndir, 4, 3, 0xF210, 0, _st())
            _lib.call("b2p_gru_lane_permute", _p(dgL), _p(dgh), B, T, H, ndir, 4, 3, 0x2F10, 0, _st())
            del dgL
        elif usemc:
            ws = _gru_mc_ws(B, H, ndir, dev)
            # frozen-parameter gradient GEMMs beside the (H/64 x 4)-CU recurrence
            _gru_bwd_launch(lambda: _lib.call("b2p_gru_bwd_mc", _p(dout), _p(whh_s), _p(out), _p(saved), _p(h0),
                                              _p(dgi), _p(dgh), _p(dh0), _p(ws), B, T, H, ndir, _st()))
            _gru_mc_fold(ws, 2, ctx.whh0, H, dev)
        else:
            dhbuf = torch.empty(ndir, B, H, device=dev)
            _gru_bwd_launch(lambda: _lib.call("b2p_gru_bwd", _p(dout), _p(whh_s), _p(out), _p(saved), _p(h0), _p(dgi),
                                              _p(dgh), _p(dh0), _p(dhbuf), B, T, H, ndir, _st()))
        grads = [None] * (4 * ndir)
        # recurrent weights: dW_hh[d] = dgh[:, :, d]^T @ hprev[d]
        hp = torch.empty(ndir, B, T, H, device=dev)
        _lib.call("b2p_gru_hprev", _p(out), _p(h0), _p(hp), B, T, H, ndir, _st())
        for d in range(ndir):
            if ctx.needs_input_grad[5 + 4 * d + 1]:
                dwhh = torch.empty(G3, H, device=dev)
                gemm(G3, H, B * T, op(dgh, d * G3, ndir * G3, False), op(hp, d * B * T * H, H, False), dwhh, H)
                grads[4 * d + 1] = dwhh
            if has_bhh and ctx.needs_input_grad[5 + 4 * d + 3]:
                db = torch.empty(G3, device=dev)
                colsum(_view_off(dgh, d * G3), B * T, G3, db, ld=ndir * G3)
                grads[4 * d + 3] = db
            if has_bih and ctx.needs_input_grad[5 + 4 * d + 2]:
                db = torch.empty(G3, device=dev)
                colsum(_view_off(dgi, d * G3), B * T, G3, db, ld=ndir * G3)
                grads[4 * d + 2] = db
        dx = None
        if ctx.implicit:
            # dgi in the padded row layout (k/s - 1 zero rows in front, L/s rows per sample, rows t >= T
            # zero): the weight gradient reads it as the k-major A operand, the input gradient as the
            # overlapping-row view (one GEMM straight into dx, no col2im)
            ktaps, stride = unf_meta
            _, L, C = x.shape
            R, lead, N3 = L // stride, ktaps // stride - 1, ndir * G3
            dgp = torch.empty((lead + B * R) * N3, device=dev, dtype=BF16)
            _lib.call("b2p_pad_rows16", _p(dgi), _p(dgp), B, T, N3, R, lead, _st())
            if any(ctx.needs_input_grad[5 + 4 * d] for d in range(ndir)):
                s16b = U16
                if s16b is None:
                    n_s, tail = B * L * C, (ktaps - stride) * C
                    s16b = torch.empty(n_s + tail, device=dev, dtype=BF16)
                    _lib.call("b2p_cast16_tail", _p(x), _p(s16b), n_s, n_s + tail, 0, _st())
                dwp = torch.empty(N3, IN, device=dev)
                gemm(N3, IN, B * R, op(dgp, lead * N3, N3, False), op(s16b, 0, stride * C, False), dwp, IN)
                del s16b
                for d in range(ndir):
                    dw = torch.empty(G3, IN, device=dev)
                    _lib.call("b2p_conv_weight_permute", _p(dwp, d * G3 * IN), _p(dw), G3, C, ktaps, 1, _st())
                    grads[4 * d] = dw
            if ctx.needs_input_grad[0]:
                dx = torch.empty(B, L, C, device=dev)
                gemm(B * R, stride * C, (ktaps // stride) * N3, op(dgp, 0, N3, True), op(wperm, 0, stride * C, False),
                     dx, stride * C)
        elif unf_meta is not None:
            ktaps, stride = unf_meta
            _, L, C = x.shape
            dgi16 = cast16(dgi) if U16 is not None else None
            if any(ctx.needs_input_grad[5 + 4 * d] for d in range(ndir)):
                dwp = torch.empty(ndir * G3, IN, device=dev)
                if U16 is not None:
                    gemm(ndir * G3, IN, B * T, op(dgi16, 0, ndir * G3, False), op(U16, 0, IN, False), dwp, IN)
                else:
                    Bop = conv_op(x, 0, C, T, L, stride, 0, C, L * C, False)
                    gemm(ndir * G3, IN, B * T, op(dgi, 0, ndir * G3, False), Bop, dwp, IN)
                for d in range(ndir):
                    dw = torch.empty(G3, IN, device=dev)
                    _lib.call("b2p_conv_weight_permute", _p(dwp, d * G3 * IN), _p(dw), G3, C, ktaps, 1, _st())
                    grads[4 * d] = dw
            if ctx.needs_input_grad[0]:
                dA = torch.empty(B * T, IN, device=dev)
                if U16 is not None:
                    gemm(B * T, IN, ndir * G3, op(dgi16, 0, ndir * G3, True), op(wperm, 0, IN, False), dA, IN)
                else:
                    gemm(B * T, IN, ndir * G3, op(dgi, 0, ndir * G3, True), op(wperm, 0, IN, False), dA, IN)
                dx = torch.empty(B, L, C, device=dev)
                _lib.call("b2p_unfold_col2im", _p(dA), None, _p(dx), B, L, C, T, ktaps, stride, _st())
        else:
            for d in range(ndir):
                if ctx.needs_input_grad[5 + 4 * d]:
                    dw = torch.empty(G3, IN, device=dev)
                    gemm(G3, IN, B * T, op(dgi, d * G3, ndir * G3, False), op(x, 0, IN, False), dw, IN)
                    grads[4 * d] = dw
            if ctx.needs_input_grad[0]:
                dx = torch.empty(B, T, IN, device=dev)
                for d in range(ndir):
                    gemm(B * T, IN, G3, op(dgi, d * G3, ndir * G3, True), op(wih[d], 0, IN, False), dx, IN,
                         beta=0.0 if d == 0 else 1.0)
        return (dx, None, None, None, dh0, *grads)


class _OffsetView:
    """Pointer + offset stand-in for the colsum helper (avoids non-contiguous torch views)."""

    def __init__(self, t, off):
        self.t, self.off = t, off

    def data_ptr(self):
        return self.t.data_ptr() + 4 * self.off


def _view_off(t, off):
    return _OffsetView(t, off)


def gru_layer(x, H, ndir, weights, h0=None):
    """One nn.GRU layer (both directions) — brain_feature_extractor.py:39-47,61-65.
    x: (B,T,IN) tensor or Unfolded; weights: [w_ih, w_hh, b_ih, b_hh] per direction.
    In the bf16x3 mode with the 'gru1' form (the Trainer policy, X3_POLICY_FORMS) the layer runs as in the
    bf16 mode (persistent MFMA recurrences, fp16 forward operands) and its backward follows it
    (_prec_follow: block 'gru'), instead of the fp32 operators' per-time-step recurrence kernels."""
    with _fp32_if("gru"):
        forms = _state.x3forms if _state.x3forms is not None else _X3_SINGLE
        ctxm = precision("bf16") if (_state.prec == 3 and "gru1" in forms) else contextlib.nullcontext()
        with ctxm:
            if isinstance(x, Unfolded):
                return _GRULayer.apply(x.src, (x.kernel, x.stride), H, ndir, h0, *weights)
            return _GRULayer.apply(x, None, H, ndir, h0, *weights)


# =====================================================================================
# Linear / dropout
# =====================================================================================
_LINEAR_DEFER = os.environ.get("B2P_LINEAR_WGRAD_DEFER", "0") == "1"   # 1: frozen Linear dW on the side stream (measured neutral: base 14.03 either way, Conformer 64.79 / 64.80 ms)


@_prec_follow
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, act):
        _chk(x, "linear.x")
        _chk(W, "linear.W")
        N, K = W.shape
        out = torch.empty(*x.shape[:-1], N, device=x.device)
        pre = torch.empty_like(out) if act else None
        mm_nt(x, W, out, bias=b, act=act, pre_out=pre)
        ctx.save_for_backward(x, W, pre)
        ctx.act = act
        ctx.has_b = b is not None
        ctx.prm = (W, b)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, W, pre = ctx.saved_tensors
        dy = dy.contiguous()
        N, K = W.shape
        if ctx.act:
            dy = _act_bwd(dy, pre, ctx.act)
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            mm_nn(dy, W, dx)
        if ctx.needs_input_grad[1]:
            if _LAZY_COLSUM and _LINEAR_DEFER and _defer_ok(ctx.prm[0]):
                # frozen weight (lm_head in configs 1-3): the weight-gradient GEMM itself on the side stream,
                # accumulating into .grad (it ran on 6 workgroups for ~47 us on the main stream)
                _defer_wgemm(ctx.prm[0], lambda out, beta, dy=dy, x=x: mm_tn(dy, x, out, beta=beta), dy, x)
            else:
                dW = torch.empty_like(W)
                mm_tn(dy, x, dW)
        if ctx.has_b and ctx.needs_input_grad[2] and not _defer_bias_rows((ctx.prm[1],), dy, dy.numel() // N, N):
            db = torch.empty(N, device=x.device)
            colsum(dy, dy.numel() // N, N, db)
        dW, db = _defer_small(ctx.prm, (dW, db))   # frozen: one batched side-stream add, not autograd's
        return dx, dW, db, None


def linear(x, W, b=None, act=0):
    with _fp32_if("linear"):
        return _Linear.apply(x.contiguous(), W, b, act)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.p, ctx.seed = p, seed
        return _dropout_raw(x.contiguous(), p, seed)

    @staticmethod
    def backward(ctx, dy):
        return _dropout_raw(dy.contiguous(), ctx.p, ctx.seed), None, None


def dropout(x, p, training):
    if not training or p <= 0.0:
        return x
    return _Dropout.apply(x, float(p), SEEDS.next())


# ------------------------------------------------------------------ LayerDrop in a captured step
def _b16_of(x):
    t = getattr(x, "_b16", None)
    return t[1] if t is not None and t[0] == x._version else None


def _h16_of(x):
    t = getattr(x, "_h16", None)
    return t[1] if t is not None and t[0] == x._version else None


class _SkipSlot:
    """The skip-path gradient of one LayerDrop-selected layer, handed from the select's backward to the
    layer Function that consumes the layer input (it adds it to its input gradient inside its last
    LayerNorm backward, b2p_layernorm_bwd_acc2, instead of autograd adding the two gradients in a
    separate pass). Exactly one of the two is nonzero (the route kernel writes dout to one side and
    zeros to the other; a skipped layer's gated backward yields exact zeros), so the sum is bitwise the
    one autograd formed."""
    __slots__ = ("claimed", "grad")

    def __init__(self):
        self.claimed = False
        self.grad = None


_SKIP_CLAIM: dict = {}   # data_ptr of a layer input -> its _SkipSlot, while that layer's forward runs
# B2P_LD_SKIP_FOLD=0: the skip gradient goes back through autograd (its own add kernel), as before
_LD_SKIP_FOLD = os.environ.get("B2P_LD_SKIP_FOLD", "1") != "0"


def _skip_claim(x):
    """Called by a layer Function's forward with its input: the slot whose skip gradient its backward
    must add to dx (None when x is not a LayerDrop-selected layer's input or was claimed already)."""
    slot = _SKIP_CLAIM.get(x.data_ptr()) if _SKIP_CLAIM else None
    if slot is None or slot.claimed:
        return None
    slot.claimed = True
    return slot


def _skip_take(slot):
    """The skip gradient for a claiming Function's backward (None: nothing to add)."""
    if slot is None:
        return None
    g, slot.grad = slot.grad, None
    return g


class _LayerDropSelect(torch.autograd.Function):
    """out = keep ? y : x with keep drawn on the device (csrc/layerdrop.hip); the backward routes
    dout to the layer (keep) or around it (skip). With a claimed _SkipSlot the skip gradient goes to
    the layer's input Function instead of back through autograd."""

    @staticmethod
    def forward(ctx, x, y, p, seed, slot=None):
        x = x.contiguous()
        y = y.contiguous()
        _chk(x, "layerdrop.x")
        _chk(y, "layerdrop.y")
        b16 = bf16_mode()
        x16, y16 = (_b16_of(x), _b16_of(y)) if b16 else (None, None)
        # the fp16 copy too when the layer made one (post-LN forward_f16): the next layer reads it uncast
        yh = _h16_of(y) if b16 and _LD_SELECT_H else None
        if _LD_INPLACE and (not b16 or y16 is not None):
            # in place: the output is a fresh tensor over y's storage (and y's 16-bit copies), overwritten
            # by x only when the replay's draw skips the layer, so a kept layer's select moves no bytes.
            # Nothing reads y's old values after a skip: the layer's own backward is gated off then.
            out = torch.empty(0, device=y.device, dtype=y.dtype).set_(y.untyped_storage(), y.storage_offset(),
                                                                       y.shape, y.stride())
            out16, outh = y16, yh
        else:
            out = torch.empty_like(y)
            out16 = torch.empty(y.shape, device=y.device, dtype=BF16) if b16 else None
            outh = torch.empty(y.shape, device=y.device, dtype=torch.float16) if yh is not None else None
        _lib.call("b2p_layerdrop_select_h", _p(x), _p(y), _p(out), _p(x16), _p(y16), _p(out16),
                  _p(_h16_of(x)) if outh is not None else None, _p(yh), _p(outh), y.numel(), float(p), seed, _st())
        ctx.p, ctx.seed, ctx.slot = p, seed, slot
        if out16 is not None:
            attach16(out, out16)
        if outh is not None:
            attach16h(out, outh)
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        d_keep = torch.empty_like(dout)
        d_skip = torch.empty_like(dout)
        _lib.call("b2p_layerdrop_route", _p(dout), _p(d_keep), _p(d_skip), dout.numel(), float(ctx.p), ctx.seed, _st())
        if ctx.slot is not None:   # folded into the layer's input gradient (_SkipSlot)
            ctx.slot.grad = d_skip
            return None, d_keep, None, None, None
        return d_skip, d_keep, None, None, None


_LD_SELECT_H = os.environ.get("B2P_LD_SELECT_H", "1") != "0"   # 0: no fp16 copy from the select (A/B)
_LD_INPLACE = os.environ.get("B2P_LD_INPLACE", "1") != "0"     # 0: the select writes a new tensor (A/B)
LAYERDROP_LOG = None   # tests: when a list, layerdrop_layer appends each layer's draw seed
# diagnostic only (B2P_GRAPH_LAYERDROP=0): a captured step keeps the host draw made at capture time
GRAPH_LAYERDROP = os.environ.get("B2P_GRAPH_LAYERDROP", "1") != "0"


def capturing() -> bool:
    """True while a step is being captured as a HIP graph: LayerDrop then draws on the device."""
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


# B2P_LAYERDROP_GATE=0: a skipped layer still computes (diagnostic / A-B of the gate)
LAYERDROP_GATE = os.environ.get("B2P_LAYERDROP_GATE", "1") != "0"
_GATE_FLAGS: list = []
# parameter id -> (weak reference, the device gate of its layer in the most recently captured step).
# HipAdam reads it while capturing: a parameter of a layer this replay dropped is left untouched, as
# torch.optim.Adam leaves a parameter whose .grad is None (the reference never ran that layer).
_LD_PARAM_GATE: dict = {}


def layerdrop_param_gates() -> dict:
    """{id(parameter): int32 device flag (1 = its layer ran in this replay)} of the last capture."""
    return {k: f for k, (r, f) in _LD_PARAM_GATE.items() if r() is not None}


def layerdrop_layer(layer, x, p):
    """One encoder layer under LayerDrop inside a captured step (see csrc/layerdrop.hip): the layer
    always runs, its output or its input is selected by the device draw of this replay, and float
    buffers it updates in place (Conformer BatchNorm running statistics) are restored when it is
    skipped. Eager steps keep the reference's host draw and skip the layer outright."""
    seed = LD_SEEDS.next()
    if LAYERDROP_LOG is not None:
        LAYERDROP_LOG.append(seed)
    bufs = [b for b in layer.buffers() if b.is_floating_point() and b.numel() % 4 == 0]
    if LAYERDROP_GATE:
        # BatchNorm running statistics are updated by bn_finalize_k, which reads the gate itself and
        # leaves them untouched in a replay that skips the layer: no snapshot / restore launches
        bn = {id(t) for m in layer.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)
              for t in (m.running_mean, m.running_var) if t is not None}
        bufs = [b for b in bufs if id(b) not in bn]
    olds = [b.clone() for b in bufs]
    y = None
    flag = torch.empty(1, dtype=torch.int32, device=x.device)
    _GATE_FLAGS.append(flag)      # referenced by the captured graph's kernels: kept for its life
    _lib.call("b2p_layerdrop_flag", _p(flag), float(p), seed, _st())
    for prm in layer.parameters():
        _LD_PARAM_GATE[id(prm)] = (weakref.ref(prm), flag)
    slot = None
    if _LD_SKIP_FOLD and LAYERDROP_GATE and x.requires_grad and x.is_contiguous():
        slot = _SkipSlot()
        _SKIP_CLAIM[x.data_ptr()] = slot
    try:
        if LAYERDROP_GATE:
            # the layer's GEMMs and fused attention (forward, backward, deferred weight gradients) read
            # this replay's draw and do no work when it skips the layer; the select below still routes
            with _gated(flag):
                y = layer(x)
        else:
            y = layer(x)
    finally:
        if slot is not None:
            _SKIP_CLAIM.pop(x.data_ptr(), None)
    for b, o in zip(bufs, olds):
        _lib.call("b2p_layerdrop_select", _p(o), _p(b), _p(b), None, None, None, b.numel(), float(p), seed, _st())
    return _LayerDropSelect.apply(x, y, float(p), seed, slot if slot is not None and slot.claimed else None)


def layerdrop_keep(p, seed, epoch=None) -> bool:
    """Host evaluation of the device draw (tests): epoch = the step counter's value in that replay."""
    k = ctypes.c_int32(0)
    _lib.check(_lib.load().b2p_layerdrop_keep(float(p), seed, 0 if epoch is None else int(epoch),
                                              0 if epoch is None else 1, ctypes.byref(k)), "b2p_layerdrop_keep")
    return bool(k.value)


# =====================================================================================
# Wav2Vec2 positional conv embedding + residual + LayerNorm + dropout
# =====================================================================================
@_prec_follow
class _PosConvLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, e, wg, wv, cbias, ln_g, ln_b, groups, eps, drop_p, seed):
        _chk(e, "pos_conv.x")
        ctx.prm = (wg, wv, cbias, ln_g, ln_b)
        B, T, D = e.shape
        O, Ig, K = wv.shape            # (D, D/groups, k)
        dev = e.device
        ws = torch.empty(int(_lib.load().b2p_weight_norm_workspace(O, Ig, K)), device=dev)
        w = torch.empty_like(wv)
        norms = torch.empty(K, device=dev)
        _lib.call("b2p_weight_norm_fwd", _p(wg), _p(wv), _p(w), _p(norms), O, Ig, K, _p(ws), _st())
        wp = torch.empty(O, K * Ig, device=dev)         # wp[o][tap*Ig + i]
        _lib.call("b2p_conv_weight_permute", _p(w), _p(wp), O, Ig, K, 0, _st())
        pre = torch.empty_like(e)
        xsum = torch.empty_like(e)
        pad = K // 2
        Og = O // groups
        fast = _posconv16_ok(B, T, D, O, Ig, K, groups)
        if fast:
            # bf16 MFMA grouped conv (csrc/posconv16.hip): slab-staged input, streamed weights
            e16 = torch.empty(B, T, D, device=dev, dtype=BF16)
            _lib.call("b2p_posconv16_fwd", _p(e), _p(cast16(wp)), _p(cbias), _p(xsum), _p(pre), _p(e16), B, T, D,
                      groups, _st())
            keep = e16
        else:
            A = conv_op(e, 0, D, T, T, 1, pad, Ig, T * D, True, bs1=Ig)
            gemm(B * T, Og, K * Ig, A, op(wp, 0, K * Ig, True, bs1=Og * K * Ig), xsum, D, cbs1=Og, nz1=groups,
                 bias=cbias, biasbs1=Og, pre_out=pre, act=ACT["gelu"], residual=e, rbs1=Og, ldr=D)
            keep = e
        if ln_g is not None:
            y, mean, rstd = _ln_fwd(xsum.view(B * T, D), ln_g, ln_b, eps, drop_p, seed)
        else:   # stable-LN encoder (TF w2v Wav2Vec2EncoderStableLayerNorm): dropout(x + pos), no LayerNorm
            y = _dropout_raw(xsum.view(B * T, D), drop_p, seed) if drop_p > 0 else xsum.view(B * T, D)
            mean = rstd = None
        ctx.save_for_backward(keep, wg, wv, w, norms, pre, xsum, ln_g, mean, rstd)
        ctx.meta = (groups, drop_p, seed, B, T, D, O, Ig, K)
        ctx.fast = fast
        return y.view(B, T, D)

    @staticmethod
    def backward(ctx, dy):
        e, wg, wv, w, norms, pre, xsum, ln_g, mean, rstd = ctx.saved_tensors
        groups, drop_p, seed, B, T, D, O, Ig, K = ctx.meta
        dev = e.device
        dy = dy.contiguous().view(B * T, D)
        if ln_g is not None:
            dxsum, dlg, dlb, _ = _ln_bwd(dy, xsum.view(B * T, D), ln_g, mean, rstd, True, None, drop_p, seed)
        else:
            dxsum = _dropout_raw(dy, drop_p, seed) if drop_p > 0 else dy
            dlg = dlb = None
        if ctx.fast:
            return _posconv16_bwd(ctx, e, wg, wv, w, norms, pre, dxsum, dlg, dlb)
        dpre = _act_bwd(dxsum, pre.view(B * T, D), ACT["gelu"])
        Og = O // groups
        pad = K // 2
        dcb = torch.empty(O, device=dev)
        colsum(dpre, B * T, D, dcb)
        dg = dv = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            # dwp[g*Og+o][tap*Ig+i] = sum_r dpre[r][g*Og+o] * e[b, t+tap-pad, g*Ig+i]
            dwp = torch.empty(O, K * Ig, device=dev)
            Bop = conv_op(e, 0, D, T, T, 1, pad, Ig, T * D, False, bs1=Ig)
            gemm(Og, K * Ig, B * T, op(dpre, 0, D, False, bs1=Og), Bop, dwp, K * Ig, cbs1=Og * K * Ig, nz1=groups)
            dw = torch.empty_like(wv)
            _lib.call("b2p_conv_weight_permute", _p(dwp), _p(dw), O, Ig, K, 1, _st())
            ws = torch.empty(int(_lib.load().b2p_weight_norm_workspace(O, Ig, K)), device=dev)
            dg = torch.empty_like(wg)
            dv = torch.empty_like(wv)
            _lib.call("b2p_weight_norm_bwd", _p(wg), _p(wv), _p(norms), _p(dw), _p(dg), _p(dv), O, Ig, K, _p(ws),
                      _st())
        de = None
        if ctx.needs_input_grad[0]:
            # de[b,s,g*Ig+i] = dxsum + sum_{k',o} dpre[b, s+k'-(K-1-pad), g*Og+o] * wt[g][i][k'*Og+o]
            wt = torch.empty(groups, Ig, K * Og, device=dev)
            _lib.call("b2p_conv_weight_transpose_flip", _p(w), _p(wt), groups, Og, Ig, K, _st())
            de = torch.empty(B, T, D, device=dev)
            A = conv_op(dpre, 0, D, T, T, 1, K - 1 - pad, Og, T * D, True, bs1=Og)
            gemm(B * T, Ig, K * Og, A, op(wt, 0, K * Og, True, bs1=Ig * K * Og), de, D, cbs1=Ig, nz1=groups,
                 residual=dxsum, rbs1=Ig, ldr=D)
        dg, dv, dcb, dlg, dlb = _defer_small(ctx.prm, (dg, dv, dcb, dlg, dlb))
        return de, dg, dv, dcb, dlg, dlb, None, None, None, None


def _posconv16_ok(B, T, D, O, Ig, K, groups) -> bool:
    return bf16_mode() and O == D and Ig == 48 and D == groups * 48 and K == 128 and 1 <= T <= 256


def _posconv16_bwd(ctx, e16, wg, wv, w, norms, pre, dxsum, dlg, dlb):
    groups, drop_p, seed, B, T, D, O, Ig, K = ctx.meta
    dev = dxsum.device
    ng = ctx.needs_input_grad
    wt = torch.empty(groups, Ig, K * (O // groups), device=dev)
    _lib.call("b2p_conv_weight_transpose_flip", _p(w), _p(wt), groups, O // groups, Ig, K, _st())
    de = torch.empty(B, T, D, device=dev)
    dpre16 = torch.empty(B, T, D, device=dev, dtype=BF16)
    part = torch.empty(B, D, device=dev)
    _lib.call("b2p_posconv16_bwd_data", _p(dxsum), _p(pre), _p(cast16(wt)), _p(de), _p(dpre16), _p(part), B, T, D,
              groups, _st())
    dcb = torch.empty(O, device=dev)
    colsum(part, B, D, dcb)
    dg = dv = None

    def wgrad():
        dwp = torch.empty(O, K * Ig, device=dev)
        _lib.call("b2p_posconv16_wgrad", _p(dpre16), _p(e16), _p(dwp), B, T, D, groups, _st())
        dw = torch.empty_like(wv)
        _lib.call("b2p_conv_weight_permute", _p(dwp), _p(dw), O, Ig, K, 1, _st())
        ws = torch.empty(int(_lib.load().b2p_weight_norm_workspace(O, Ig, K)), device=dev)
        g_, v_ = torch.empty_like(wg), torch.empty_like(wv)
        _lib.call("b2p_weight_norm_bwd", _p(wg), _p(wv), _p(norms), _p(dw), _p(g_), _p(v_), O, Ig, K, _p(ws), _st())
        return g_, v_

    if ng[1] and ng[2] and _LAZY_COLSUM and _defer_ok(ctx.prm[0]) and _defer_ok(ctx.prm[1]):
        # frozen weight-normed pos-conv: its weight gradient (conv wgrad, permute, weight-norm backward)
        # runs on the side stream and joins the flush's batched accumulation
        def run():
            g_, v_ = wgrad()
            _defer_acc(ctx.prm[0], g_)
            _defer_acc(ctx.prm[1], v_)
        _Deferred.queue.append((_gate_wrap(run), (dpre16, e16, norms), id(ctx.prm[0]), None))
    elif ng[1] or ng[2]:
        dg, dv = wgrad()
    # frozen parameters' gradients join the batched side-stream accumulation (no autograd adds)
    dg, dv, dcb, dlg, dlb = _defer_small(ctx.prm, (dg, dv, dcb, dlg, dlb))
    return (de if ng[0] else None), dg, dv, dcb, dlg, dlb, None, None, None, None


def pos_conv_ln(e, wg, wv, cbias, ln_g, ln_b, groups, eps, drop_p, training):
    """dropout(LN(e + gelu(posconv(e)))); ln_g = ln_b = None: dropout(e + gelu(posconv(e))) (stable-LN)."""
    p = drop_p if training else 0.0
    seed = SEEDS.next() if p > 0 else 0
    with _fp32_if("posconv"):
        return _PosConvLN.apply(e.contiguous(), wg, wv, cbias, ln_g, ln_b, groups, eps, p, seed)


# =====================================================================================
# attention core shared by the w2v and Conformer layers: softmax(Q K^T * scale) -> dropout -> @ V
# qkv (B*T, 3D) laid out [b][t][q|k|v][h][dh]
# =====================================================================================
def _attn_core_fwd(qkv, B, T, nh, dh, p_attn, seed, want16=False):
    D = nh * dh
    dev = qkv.device
    Tp = (T + 3) // 4 * 4
    S = torch.empty(B, nh, T, Tp, device=dev)
    gemm(T, T, dh, op(qkv, 0, 3 * D, True, bs1=T * 3 * D, bs2=dh), op(qkv, D, 3 * D, True, bs1=T * 3 * D, bs2=dh),
         S, Tp, cbs1=nh * T * Tp, cbs2=T * Tp, nz1=B, nz2=nh, alpha=dh ** -0.5)
    P = torch.empty_like(S)
    Pd = torch.empty_like(S) if p_attn > 0 else P
    _lib.call("b2p_softmax_fwd", _p(S), _p(P), _p(Pd), B * nh * T, T, Tp, float(p_attn), seed, _st())
    del S
    O = torch.empty(B * T, D, device=dev)
    O16 = torch.empty(B * T, D, device=dev, dtype=BF16) if want16 else None
    gemm(T, dh, T, op(Pd, 0, Tp, True, bs1=nh * T * Tp, bs2=T * Tp),
         op(qkv, 2 * D, 3 * D, False, bs1=T * 3 * D, bs2=dh), O, D, cbs1=T * D, cbs2=dh, nz1=B, nz2=nh, C16=O16)
    if want16:
        return P, (Pd if p_attn > 0 else None), O, O16
    return P, (Pd if p_attn > 0 else None), O


def _attn_core_bwd(qkv, P, Pd, dO, B, T, nh, dh, p_attn, seed, want16=False):
    """returns dqkv (B*T, 3D) = [dQ | dK | dV] (and its bf16 copy when want16)"""
    D = nh * dh
    dev = qkv.device
    Tp = P.shape[-1]
    Pd = P if Pd is None else Pd
    scale = dh ** -0.5
    dPd = torch.empty(B, nh, T, Tp, device=dev)
    gemm(T, T, dh, op(dO, 0, D, True, bs1=T * D, bs2=dh), op(qkv, 2 * D, 3 * D, True, bs1=T * 3 * D, bs2=dh),
         dPd, Tp, cbs1=nh * T * Tp, cbs2=T * Tp, nz1=B, nz2=nh)
    dqkv = torch.empty(B * T, 3 * D, device=dev)
    d16 = torch.empty(B * T, 3 * D, device=dev, dtype=BF16) if want16 else None
    gemm(T, dh, T, op(Pd, 0, Tp, False, bs1=nh * T * Tp, bs2=T * Tp), op(dO, 0, D, False, bs1=T * D, bs2=dh),
         dqkv, 3 * D, c_off=2 * D, cbs1=T * 3 * D, cbs2=dh, nz1=B, nz2=nh, C16=d16)
    dS = torch.empty_like(dPd)
    _lib.call("b2p_softmax_bwd", _p(P), _p(dPd), _p(dS), B * nh * T, T, Tp, float(p_attn), seed, _st())
    del dPd
    gemm(T, dh, T, op(dS, 0, Tp, True, bs1=nh * T * Tp, bs2=T * Tp),
         op(qkv, D, 3 * D, False, bs1=T * 3 * D, bs2=dh), dqkv, 3 * D, c_off=0, cbs1=T * 3 * D, cbs2=dh,
         nz1=B, nz2=nh, alpha=scale, C16=d16)
    gemm(T, dh, T, op(dS, 0, Tp, False, bs1=nh * T * Tp, bs2=T * Tp),
         op(qkv, 0, 3 * D, False, bs1=T * 3 * D, bs2=dh), dqkv, 3 * D, c_off=D, cbs1=T * 3 * D, cbs2=dh,
         nz1=B, nz2=nh, alpha=scale, C16=d16)
    if want16:
        return dqkv, d16
    return dqkv


def attn16_ok(T, dh) -> bool:
    """The fused bf16 attention kernels (csrc/attn16.hip) cover head size 64 and T' <= 512 (windows of up
    to 2,080 bins; the 256-key class keeps the dropout keep bits for the backward, the 512-key class
    rehashes them)."""
    return dh == 64 and 0 < T <= 512


# ---------------------------------------------------------------- attention keep masks drawn ahead
# The attention dropout keep bits of every layer of one encoder forward, drawn by one launch
# (b2p_attn16_keep_masks) on a side stream at the start of the model's forward (beside the front end);
# each layer's fused attention forward then reads its bits
# (b2p_attn16_fwd[_f16]_keep) instead of hashing them inside its VALU-bound softmax loop, and the
# backward reads the same block as before. Layers take the blocks in call order (a host-skipped
# LayerDrop layer leaves one unused: every block is an independent draw). Measured: attention forward
# 38.4 -> 33.2 us per base layer, the step unchanged within noise (profiles/r05ag_attn_keep_ahead_ab.txt).
# B2P_ATTN_KEEP_AHEAD=0: each forward hashes its own (A/B).
_KEEP_AHEAD = [os.environ.get("B2P_ATTN_KEEP_AHEAD", "1") != "0"]
_KEEP_PLAN: list = [None]


class _KeepPlan:
    def __init__(self, n, B, T, nh, p):
        self.key = (B, T, nh, float(p))
        self.n, self.next, self.joined, self.ev = n, 0, False, None
        self.masks = torch.empty(n, B, nh, T, 8, device=torch.cuda.current_stream().device, dtype=torch.int32)
        self.seeds = (ctypes.c_uint64 * n)(*[SEEDS.next() for _ in range(n)])

    def launch(self) -> None:
        """Issue the draw on the side stream, ordered after the main stream's work so far. Issued at the
        start of the model forward it runs beside the front end (profiles/r05ag_attn_keep_ahead_ab.txt:
        issued at the GRU recurrence's launch instead, it slowed the 4-CU recurrence by 20 %)."""
        if self.ev is not None:
            return
        main = torch.cuda.current_stream()
        if not _Deferred.sides:
            n_side = max(1, int(os.environ.get("B2P_SIDE_STREAMS", "1")))
            _Deferred.sides = [torch.cuda.Stream(device=main.device) for _ in range(n_side)]
        side = main if SERIAL_SIDE else _Deferred.sides[0]
        B, T, nh, p = self.key
        side.wait_stream(main)
        with torch.cuda.stream(side):
            _lib.call("b2p_attn16_keep_masks", _p(self.masks), ctypes.addressof(self.seeds), self.n, B, T, nh, p,
                      _st())
            self.ev = torch.cuda.Event()
            self.ev.record()
        self.masks.record_stream(side)

    def join(self) -> None:
        if not self.joined:
            self.launch()
            torch.cuda.current_stream().wait_event(self.ev)
            self.joined = True

    def take(self, B, T, nh, p):
        if (B, T, nh, float(p)) != self.key or self.next >= self.n:
            return None
        self.join()
        self.next += 1
        return self.masks[self.next - 1]


@contextlib.contextmanager
def attn_keep_plan(n_layers, B, T, nh, dh, p_attn, training):
    """Around a model forward: draw the encoder's attention keep masks ahead (see _KeepPlan) when the
    fused 16-bit attention with a stored mask will run (bf16 mode, training, p > 0, T' <= 256)."""
    on = (_KEEP_AHEAD[0] and training and p_attn > 0 and n_layers > 0 and bf16_mode()
          and attn16_ok(T, dh) and T <= 256 and _KEEP_PLAN[0] is None)
    if not on:
        yield
        return
    _KEEP_PLAN[0] = _KeepPlan(int(n_layers), int(B), int(T), int(nh), p_attn)
    _KEEP_PLAN[0].launch()
    try:
        yield
    finally:
        pl, _KEEP_PLAN[0] = _KEEP_PLAN[0], None
        pl.join()   # a capture must join the side stream even when no layer took a block


def attn_keep_plan_cfg(cfg, brain_encoder, inputs, training):
    """attn_keep_plan for an encoder config (num_hidden_layers, num_attention_heads, hidden_size,
    attention_dropout) and the brain encoder's input (B, L, ...): the encoder sees T' =
    brain_encoder.output_length(L) frames (the B2P2T Unfold; the GRU keeps the length)."""
    shp = getattr(inputs, "shape", None)
    if shp is None or len(shp) < 2:
        return contextlib.nullcontext()
    T = brain_encoder.output_length(shp[1]) if hasattr(brain_encoder, "output_length") else shp[1]
    return attn_keep_plan(cfg.num_hidden_layers, shp[0], T, cfg.num_attention_heads,
                          cfg.hidden_size // cfg.num_attention_heads, cfg.attention_dropout, training)


# Where the queued frozen weight gradients go out relative to the GRU recurrence backward (A/B):
# "after" = flushed after the recurrence launch, ordered after the event before it; "first" = flushed
# before the recurrence launch; "fork" = the recurrence itself launched on a stream of its own (forked
# from and joined back into the current stream), the flush after it. All three measured equal step
# times (base 14.49 / 14.49 / 14.47 ms, Conformer 66.11 / - / 65.96 ms: profiles/r05ak_gru_bwd_mode_ab.txt).
_GRU_BWD_MODE = os.environ.get("B2P_GRU_BWD_MODE", "after")
_GRU_STREAM: list = [None]


def _gru_bwd_launch(launch) -> None:
    """Launch a GRU recurrence backward (launch() on the current stream) with the frozen weight
    gradients flushed beside it (flush_wgrad), in the order _GRU_BWD_MODE selects."""
    ev = torch.cuda.Event()
    ev.record()
    if _GRU_BWD_MODE == "first":
        flush_wgrad(ev)
        launch()
    elif _GRU_BWD_MODE == "fork":
        main = torch.cuda.current_stream()
        if _GRU_STREAM[0] is None:
            _GRU_STREAM[0] = torch.cuda.Stream(device=main.device)
        gs = _GRU_STREAM[0]
        gs.wait_event(ev)
        with torch.cuda.stream(gs):
            launch()
            done = torch.cuda.Event()
            done.record()
        flush_wgrad(ev)
        main.wait_event(done)
    else:
        launch()
        flush_wgrad(ev)


def _keep_take(B, T, nh, p_attn):
    pl = _KEEP_PLAN[0]
    return None if pl is None or p_attn <= 0 else pl.take(B, T, nh, p_attn)


def _attn16_fwd(qkv16, B, T, nh, dh, p_attn, seed, want_mask=False):
    """qkv16 (B*T, 3D) bf16 -> O16 (B*T, D) bf16, lse2 (B, nh, T) f32 (fused, scores stay on-chip)
    [, mask: the dropout keep bits (B, nh, T, 8) int32 for the backward, None without dropout]."""
    dev = qkv16.device
    O16 = torch.empty(B * T, nh * dh, device=dev, dtype=BF16)
    lse2 = torch.empty(B, nh, T, device=dev)
    mask = _keep_take(B, T, nh, p_attn) if want_mask else None
    if mask is not None:
        _lib.call("b2p_attn16_fwd_keep", _p(qkv16), _p(O16), _p(lse2), B, T, nh, dh, float(dh ** -0.5),
                  float(p_attn), mask.data_ptr(), _st())
        return O16, lse2, mask
    # the stored keep mask covers T' <= 256 (32 bytes a row); longer windows rehash in the backward
    mask = torch.empty(B, nh, T, 8, device=dev, dtype=torch.int32) if (want_mask and p_attn > 0 and T <= 256) else None
    _lib.call("b2p_attn16_fwd", _p(qkv16), _p(O16), _p(lse2), B, T, nh, dh, float(dh ** -0.5), float(p_attn),
              seed, None if mask is None else mask.data_ptr(), _st())
    return (O16, lse2, mask) if want_mask else (O16, lse2)


# bf16 precision mode: the fused attention's forward operands (Q, K, V, the probabilities, O) in fp16
# (csrc/attn16.hip b2p_attn16_fwd_f16). bf16's 8-bit mantissa on the scores / probabilities biased the
# 24-layer models' CTC loss by ~1e-3 relative (tools/fixture_err.py: with the attention alone in exact
# fp32 the Conformer-large error fell from 1.0e-3 to 8e-5). The QKV projection writes the fp16 operand,
# the backward recomputes the scores from it (b2p_attn16_bwd_f16); B2P_ATTN_F16=0 keeps bf16 (A/B).
ATTN_F16 = os.environ.get("B2P_ATTN_F16", "1") != "0"


def _attn16_fwd_f16(qkvh, B, T, nh, dh, p_attn, seed):
    """qkvh (B*T, 3D) fp16 -> Oh (B*T, D) fp16 (the out-projection's operand), Ob (B*T, D) bf16 (its
    weight-gradient operand), lse2 (B, nh, T) f32, the dropout keep bits (None without dropout)."""
    dev = qkvh.device
    Oh = torch.empty(B * T, nh * dh, device=dev, dtype=torch.float16)
    Ob = torch.empty(B * T, nh * dh, device=dev, dtype=BF16)
    lse2 = torch.empty(B, nh, T, device=dev)
    mask = _keep_take(B, T, nh, p_attn)
    if mask is not None:
        _lib.call("b2p_attn16_fwd_f16_keep", _p(qkvh), _p(Oh), _p(Ob), _p(lse2), B, T, nh, dh, float(dh ** -0.5),
                  float(p_attn), mask.data_ptr(), _st())
        return Oh, Ob, lse2, mask
    mask = torch.empty(B, nh, T, 8, device=dev, dtype=torch.int32) if (p_attn > 0 and T <= 256) else None
    _lib.call("b2p_attn16_fwd_f16", _p(qkvh), _p(Oh), _p(Ob), _p(lse2), B, T, nh, dh, float(dh ** -0.5),
              float(p_attn), seed, None if mask is None else mask.data_ptr(), _st())
    return Oh, Ob, lse2, mask


def _attn16_bwd(qkv16, dO16, lse2, B, T, nh, dh, p_attn, seed, want32=True, mask=None):
    """-> dqkv (B*T, 3D) f32 (or None) and its bf16 copy (mask: the forward's keep bits, or None to
    re-hash). qkv16 fp16 (the _attn16_fwd_f16 forward) selects b2p_attn16_bwd_f16."""
    dev = qkv16.device
    dqkv = torch.empty(B * T, 3 * nh * dh, device=dev) if want32 else None
    d16 = torch.empty(B * T, 3 * nh * dh, device=dev, dtype=BF16)
    delta = torch.empty(B, nh, T, device=dev)
    fn = "b2p_attn16_bwd_f16" if qkv16.dtype == torch.float16 else "b2p_attn16_bwd"
    _lib.call(fn, _p(qkv16), _p(dO16), _p(lse2), _p(delta), _p(dqkv), _p(d16), B, T, nh, dh,
              float(dh ** -0.5), float(p_attn), seed, None if mask is None else mask.data_ptr(), _st())
    return dqkv, d16


# =====================================================================================
# post-LN transformer encoder layer (Wav2Vec2EncoderLayer)
# =====================================================================================
@_gate_aware
@_prec_follow
class _EncoderLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cfg, wq, bq, wk, bk, wv, bv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2):
        ctx.skip = _skip_claim(x)   # LayerDrop skip gradient folded into dx (_SkipSlot)
        nh, eps, p_attn, p_hid, p_act, seeds = cfg
        _chk(x, "encoder_layer.x")
        B, T, D = x.shape
        dh = D // nh
        NT = B * T
        F = w1.shape[0]
        dev = x.device
        x2 = x.view(NT, D)
        qkv = torch.empty(NT, 3 * D, device=dev)
        for i, (w, b) in enumerate(((wq, bq), (wk, bk), (wv, bv))):
            gemm(NT, D, D, op(x2, 0, D, True), op(w, 0, D, True), qkv, 3 * D, c_off=i * D, bias=b)
        P, Pd, O = _attn_core_fwd(qkv, B, T, nh, dh, p_attn, seeds[0])
        # y1 = x + dropout(O Wo^T + bo)
        y1 = torch.empty(NT, D, device=dev)
        gemm(NT, D, D, op(O, 0, D, True), op(wo, 0, D, True), y1, D, bias=bo, drop_p=p_hid, seed=seeds[1],
             residual=x2)
        x1, m1, r1 = _ln_fwd(y1, g1, be1, eps)
        # FFN: f = dropout(gelu(x1 W1^T + b1)); y2 = x1 + dropout(f W2^T + b2)
        pre = torch.empty(NT, F, device=dev)
        f = torch.empty(NT, F, device=dev)
        gemm(NT, F, D, op(x1, 0, D, True), op(w1, 0, D, True), f, F, bias=b1, pre_out=pre, act=ACT["gelu"],
             drop_p=p_act, seed=seeds[2])
        y2 = torch.empty(NT, D, device=dev)
        gemm(NT, D, F, op(f, 0, F, True), op(w2, 0, F, True), y2, D, bias=b2, drop_p=p_hid, seed=seeds[3],
             residual=x1)
        out, m2, r2 = _ln_fwd(y2, g2, be2, eps)
        ctx.save_for_backward(x, qkv, P, Pd, O, y1, x1, m1, r1, pre, f, y2, m2, r2,
                              wq, wk, wv, wo, g1, w1, w2, g2)
        ctx.cfg = cfg
        ctx.has_b = [b is not None for b in (bq, bk, bv, bo, b1, b2)]
        return out.view(B, T, D)

    @staticmethod
    def backward(ctx, dout):
        (x, qkv, P, Pd, O, y1, x1, m1, r1, pre, f, y2, m2, r2, wq, wk, wv, wo, g1, w1, w2, g2) = ctx.saved_tensors
        nh, eps, p_attn, p_hid, p_act, seeds = ctx.cfg
        B, T, D = x.shape
        dh = D // nh
        NT = B * T
        F = w1.shape[0]
        dev = x.device
        Tp = P.shape[-1]
        scale = dh ** -0.5
        ng = ctx.needs_input_grad
        dout = dout.contiguous().view(NT, D)
        x2 = x.view(NT, D)
        # LN2 backward -> dy2 ; dz2 = dropout-mask(dy2) (output dropout of the FFN)
        db2 = torch.empty(D, device=dev) if ng[15] else None
        dy2, dg2, dbe2, dz2 = _ln_bwd(dout, y2, g2, m2, r2, True, in_drop_p=p_hid, in_seed=seeds[3], dbias_in=db2)
        dw2 = torch.empty_like(w2) if ng[14] else None
        if dw2 is not None:
            mm_tn(dz2, f, dw2)
        # dpre = (dz2 W2) * mask_act * gelu'(pre)
        dpre = torch.empty(NT, F, device=dev)
        gemm(NT, F, D, op(dz2, 0, D, True), op(w2, 0, F, False), dpre, F, drop_p=p_act, seed=seeds[2],
             act_bwd=ACT["gelu"], aux=pre)
        dw1 = torch.empty_like(w1) if ng[12] else None
        if dw1 is not None:
            mm_tn(dpre, x1, dw1)
        db1 = torch.empty(F, device=dev) if ng[13] else None
        if db1 is not None:
            colsum(dpre, NT, F, db1)
        # dx1 = dpre W1 + dy2
        dx1 = torch.empty(NT, D, device=dev)
        gemm(NT, D, F, op(dpre, 0, F, True), op(w1, 0, D, False), dx1, D, residual=dy2)
        del dpre
        # LN1 backward -> dy1 ; dz1 = dropout-mask(dy1) (attention output dropout)
        dbo = torch.empty(D, device=dev) if ng[9] else None
        dy1, dg1, dbe1, dz1 = _ln_bwd(dx1, y1, g1, m1, r1, True, in_drop_p=p_hid, in_seed=seeds[1], dbias_in=dbo,
                                       dx_accum2=_skip_take(ctx.skip))
        dwo = torch.empty_like(wo) if ng[8] else None
        if dwo is not None:
            mm_tn(dz1, O, dwo)
        dO = torch.empty(NT, D, device=dev)
        mm_nn(dz1, wo, dO)
        dqkv = _attn_core_bwd(qkv, P, Pd, dO, B, T, nh, dh, p_attn, seeds[0])
        grads_w = []
        for i, w in enumerate((wq, wk, wv)):
            gw = gb = None
            if ng[2 + 2 * i]:
                gw = torch.empty_like(w)
                gemm(D, D, NT, op(dqkv, i * D, 3 * D, False), op(x2, 0, D, False), gw, D)
            if ctx.has_b[i] and ng[3 + 2 * i]:
                gb = torch.empty(D, device=dev)
                colsum(_view_off(dqkv, i * D), NT, D, gb, ld=3 * D)
            grads_w += [gw, gb]
        dx = None
        if ng[0]:
            dx = torch.empty(NT, D, device=dev)
            for i, w in enumerate((wq, wk, wv)):
                gemm(NT, D, D, op(dqkv, i * D, 3 * D, True), op(w, 0, D, False), dx, D,
                     residual=dy1 if i == 0 else None, beta=0.0 if i == 0 else 1.0)
            dx = dx.view(B, T, D)
        return (dx, None, *grads_w, dwo, dbo, dg1, dbe1, dw1, db1, dw2, db2, dg2, dbe2)


@_gate_aware
@_prec_follow
class _EncoderLayer16(torch.autograd.Function):
    """bf16-operand variant of _EncoderLayer (same math, same dropout masks): Q/K/V fused into one
    GEMM over the concatenated bf16 weight, every projection reading bf16 copies written by the
    producing kernel; fp32 residual stream, LayerNorm statistics and gradients."""

    @staticmethod
    def forward(ctx, x, cfg, wq, bq, wk, bk, wv, bv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2):
        ctx.skip = _skip_claim(x)   # LayerDrop skip gradient folded into dx (_SkipSlot)
        nh, eps, p_attn, p_hid, p_act, seeds = cfg
        _chk(x, "encoder_layer.x")
        B, T, D = x.shape
        dh = D // nh
        NT = B * T
        F = w1.shape[0]
        dev = x.device
        x2 = x.view(NT, D)
        x16 = to16(x).view(NT, D)
        bqkv = bias_cat(bq, bk, bv) if any(b is not None for b in (bq, bk, bv)) else None
        fused = attn16_ok(T, dh)
        if fused and ATTN_F16 and _state.fwd16:
            return _EncoderLayer16._forward_f16(ctx, x, x16, cfg, bqkv, B, T, D, nh, dh, wq, bq, wk, bk, wv, bv, wo,
                                                bo, g1, be1, w1, b1, w2, b2, g2, be2)
        wqkv16 = weight16(wq, wk, wv)
        Oh = None
        if fused:
            if ATTN_F16:   # fp16 attention operand (the saved qkv: the backward recomputes from it)
                qkv = torch.empty(NT, 3 * D, device=dev, dtype=torch.float16)
                gemm(NT, 3 * D, D, op(x16, 0, D, True), op(wqkv16, 0, D, True), None, 3 * D, bias=bqkv, C16=qkv,
                     c16_fp16=True)
                Oh, O16, P, Pd = _attn16_fwd_f16(qkv, B, T, nh, dh, p_attn, seeds[0])
            else:
                qkv = torch.empty(NT, 3 * D, device=dev, dtype=BF16)     # bf16 only: attention operand
                gemm(NT, 3 * D, D, op(x16, 0, D, True), op(wqkv16, 0, D, True), None, 3 * D, bias=bqkv, C16=qkv)
                # P slot: lse2, Pd slot: the dropout keep bits for the backward
                O16, P, Pd = _attn16_fwd(qkv, B, T, nh, dh, p_attn, seeds[0], want_mask=True)
        else:
            qkv = torch.empty(NT, 3 * D, device=dev)
            gemm(NT, 3 * D, D, op(x16, 0, D, True), op(wqkv16, 0, D, True), qkv, 3 * D, bias=bqkv)
            P, Pd, _O, O16 = _attn_core_fwd(qkv, B, T, nh, dh, p_attn, seeds[0], want16=True)
            del _O
        # y1 = x + dropout(O Wo^T + bo)   (fp16 O: the fp16 weight copy)
        wo16, wo_op = _w_op16(wo, Oh is not None)
        y1 = torch.empty(NT, D, device=dev)
        gemm(NT, D, D, op(O16 if Oh is None else Oh, 0, D, True), wo_op, y1, D, bias=bo, drop_p=p_hid,
             seed=seeds[1], residual=x2)
        del Oh, wo16
        x1, x1_16, m1, r1 = _ln_fwd16(y1, g1, be1, eps)
        # FFN: f = dropout(gelu(x1 W1^T + b1)) (bf16 only: it is a GEMM operand and nothing else)
        w1_16, w2_16 = weight16(w1), weight16(w2)
        pre = torch.empty(NT, F, device=dev, dtype=BF16)      # bf16 pre-activation: GELU' operand
        f16 = torch.empty(NT, F, device=dev, dtype=BF16)
        gemm(NT, F, D, op(x1_16, 0, D, True), op(w1_16, 0, D, True), None, F, bias=b1, pre16=pre,
             act=ACT["gelu"], drop_p=p_act, seed=seeds[2], C16=f16)
        y2 = torch.empty(NT, D, device=dev)
        gemm(NT, D, F, op(f16, 0, F, True), op(w2_16, 0, F, True), y2, D, bias=b2, drop_p=p_hid, seed=seeds[3],
             residual=x1)
        del x1
        out, out16, m2, r2 = _ln_fwd16(y2, g2, be2, eps)
        ctx.save_for_backward(x16, qkv, P, Pd, O16, y1, x1_16, m1, r1, pre, f16, y2, m2, r2,
                              wq, wk, wv, wo, g1, w1, w2, g2)
        ctx.cfg = cfg
        ctx.shape = (B, T, D)
        ctx.fused = fused
        ctx.prm = (wq, bq, wk, bk, wv, bv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2)
        ctx.has_b = [b is not None for b in (bq, bk, bv, bo, b1, b2)]
        res = out.view(B, T, D)
        attach16(res, out16.view(B, T, D))
        return res

    @staticmethod
    def _forward_f16(ctx, x, x16, cfg, bqkv, B, T, D, nh, dh, wq, bq, wk, bk, wv, bv, wo, bo, g1, be1, w1, b1, w2, b2,
                     g2, be2):
        """forward_f16: every GEMM operand of the layer in fp16 (the QKV, out-projection and FFN inputs and
        weights; 11 significant bits instead of bf16's 8, same MFMA rate). The producers write the
        backward's bf16 operands beside the fp16 ones (LayerNorm: y16b; FFN1 epilogue: C16b; attention:
        Ob), so the backward is the bf16 one, unchanged."""
        nh, eps, p_attn, p_hid, p_act, seeds = cfg
        NT = B * T
        F = w1.shape[0]
        dev = x.device
        x2 = x.view(NT, D)
        xh = to16h(x).view(NT, D)
        qkv = torch.empty(NT, 3 * D, device=dev, dtype=torch.float16)
        gemm(NT, 3 * D, D, op(xh, 0, D, True), op(weight16(wq, wk, wv, half=True), 0, D, True), None, 3 * D,
             bias=bqkv, C16=qkv, c16_fp16=True)
        Oh, O16, P, Pd = _attn16_fwd_f16(qkv, B, T, nh, dh, p_attn, seeds[0])
        y1 = torch.empty(NT, D, device=dev)
        gemm(NT, D, D, op(Oh, 0, D, True), op(weight16(wo, half=True), 0, D, True), y1, D, bias=bo, drop_p=p_hid,
             seed=seeds[1], residual=x2)
        del Oh
        x1, x1h, m1, r1, x1_16 = _ln_fwd_x16(y1, g1, be1, eps, True, want32=True, want_b16=True)
        pre = torch.empty(NT, F, device=dev, dtype=BF16)        # bf16 pre-activation: GELU' operand
        fh = torch.empty(NT, F, device=dev, dtype=torch.float16)
        f16 = torch.empty(NT, F, device=dev, dtype=BF16)       # the dW2 operand
        gemm(NT, F, D, op(x1h, 0, D, True), op(weight16(w1, half=True), 0, D, True), None, F, bias=b1, pre16=pre,
             act=ACT["gelu"], drop_p=p_act, seed=seeds[2], C16=fh, c16_fp16=True, C16b=f16)
        del x1h
        y2 = torch.empty(NT, D, device=dev)
        gemm(NT, D, F, op(fh, 0, F, True), op(weight16(w2, half=True), 0, F, True), y2, D, bias=b2, drop_p=p_hid,
             seed=seeds[3], residual=x1)
        del x1, fh
        out, outh, m2, r2, out16 = _ln_fwd_x16(y2, g2, be2, eps, True, want32=True, want_b16=True)
        ctx.save_for_backward(x16, qkv, P, Pd, O16, y1, x1_16, m1, r1, pre, f16, y2, m2, r2,
                              wq, wk, wv, wo, g1, w1, w2, g2)
        ctx.cfg = cfg
        ctx.shape = (B, T, D)
        ctx.fused = True
        ctx.prm = (wq, bq, wk, bk, wv, bv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2)
        ctx.has_b = [b is not None for b in (bq, bk, bv, bo, b1, b2)]
        res = out.view(B, T, D)
        attach16(res, out16.view(B, T, D))
        attach16h(res, outh.view(B, T, D))
        return res

    @staticmethod
    def backward(ctx, dout):
        (x16, qkv, P, Pd, O16, y1, x1_16, m1, r1, pre, f16, y2, m2, r2, wq, wk, wv, wo, g1, w1, w2,
         g2) = ctx.saved_tensors
        nh, eps, p_attn, p_hid, p_act, seeds = ctx.cfg
        B, T, D = ctx.shape
        dh = D // nh
        NT = B * T
        F = w1.shape[0]
        dev = y1.device
        ng = ctx.needs_input_grad
        dout = dout.contiguous().view(NT, D)
        # transposed bf16 weights: every backward-data GEMM runs on the k-contiguous (NT) kernel
        w1t16, w2t16, wot16, wqkvt16 = weight16t(w1), weight16t(w2), weight16t(wo), weight16t(wq, wk, wv)
        # LN2 backward -> dy2 ; dz2 = dropout-mask(dy2) (output dropout of the FFN), bf16 copy dz2_16
        db2 = torch.empty(D, device=dev) if ng[15] else None
        prm = ctx.prm
        dy2, dg2, dbe2, _dz2, dz2_16, db2 = _ln_bwd16(dout, y2, g2, m2, r2, True, in_drop_p=p_hid, in_seed=seeds[3],
                                                      dbias_in=db2, lazy=(prm[14], prm[15], prm[13] if ng[15] else None))
        del _dz2
        dw2 = None
        if ng[14]:
            if _defer_ok(w2):
                _defer_wspec((prm[12],), D, F, NT, dz2_16, 0, D, f16, F)
            else:
                dw2 = torch.empty_like(w2)
                gemm(D, F, NT, op(dz2_16, 0, D, False), op(f16, 0, F, False), dw2, F)
        # dpre = (dz2 W2) * mask_act * gelu'(pre): bf16 for the GEMMs; its column sums (the FFN1 bias
        # gradient) are reduced inside the epilogue from the fp32 values
        dpre16 = torch.empty(NT, F, device=dev, dtype=BF16)
        parts = colsum_parts_buf(NT, F, dev) if ng[13] else None
        gemm(NT, F, D, op(dz2_16, 0, D, True), op(w2t16, 0, D, True), None, F, drop_p=p_act, seed=seeds[2],
             act_bwd=ACT["gelu"], aux16=pre, C16=dpre16, colsum_part=parts)
        dw1 = None
        if ng[12]:
            if _defer_ok(w1):
                _defer_wspec((prm[10],), F, D, NT, dpre16, 0, F, x1_16, D)
            else:
                dw1 = torch.empty_like(w1)
                gemm(F, D, NT, op(dpre16, 0, F, False), op(x1_16, 0, D, False), dw1, D)
        db1 = ColsumParts(parts) if ng[13] else None   # finished below (deferred) or materialised
        # dx1 = dpre W1 + dy2
        dx1 = torch.empty(NT, D, device=dev)
        gemm(NT, D, F, op(dpre16, 0, F, True), op(w1t16, 0, F, True), dx1, D, residual=dy2)
        del dpre16
        # LN1 backward -> dy1 ; dz1 = dropout-mask(dy1) (attention output dropout)
        dbo = torch.empty(D, device=dev) if ng[9] else None
        dy1, dg1, dbe1, _dz1, dz1_16, dbo = _ln_bwd16(dx1, y1, g1, m1, r1, True, in_drop_p=p_hid, in_seed=seeds[1],
                                                      dbias_in=dbo, dx_accum2=_skip_take(ctx.skip),
                                                      lazy=(prm[8], prm[9], prm[7] if ng[9] else None))
        del _dz1
        dwo = None
        if ng[8]:
            if _defer_ok(wo):
                _defer_wspec((prm[6],), D, D, NT, dz1_16, 0, D, O16, D)
            else:
                dwo = torch.empty_like(wo)
                gemm(D, D, NT, op(dz1_16, 0, D, False), op(O16, 0, D, False), dwo, D)
        if ctx.fused:
            dO16 = torch.empty(NT, D, device=dev, dtype=BF16)
            gemm(NT, D, D, op(dz1_16, 0, D, True), op(wot16, 0, D, True), None, D, C16=dO16)
            dqkv, dqkv16 = _attn16_bwd(qkv, dO16, P, B, T, nh, dh, p_attn, seeds[0], mask=Pd)
            del dO16
        else:
            dO = torch.empty(NT, D, device=dev)
            gemm(NT, D, D, op(dz1_16, 0, D, True), op(wot16, 0, D, True), dO, D)
            dqkv, dqkv16 = _attn_core_bwd(qkv, P, Pd, dO, B, T, nh, dh, p_attn, seeds[0], want16=True)
            del dO
        grads_w = [None] * 6
        if all(_defer_ok(w) for w in (wq, wk, wv)) and ng[2] and ng[4] and ng[6]:
            _defer_wspec((prm[0], prm[2], prm[4]), 3 * D, D, NT, dqkv16, 0, 3 * D, x16, D)
        elif ng[2] or ng[4] or ng[6]:
            dwqkv = torch.empty(3 * D, D, device=dev)
            gemm(3 * D, D, NT, op(dqkv16, 0, 3 * D, False), op(x16, 0, D, False), dwqkv, D)
            for i in range(3):
                if ng[2 + 2 * i]:
                    grads_w[2 * i] = dwqkv[i * D:(i + 1) * D]
        if all(ctx.has_b[i] and ng[3 + 2 * i] for i in range(3)) and _defer_bias_rows((prm[1], prm[3], prm[5]), dqkv, NT,
                                                                                        3 * D):
            pass   # frozen Q/K/V biases: their column sums run on the side stream
        elif any(ctx.has_b[i] and ng[3 + 2 * i] for i in range(3)):
            dbqkv = torch.empty(3 * D, device=dev)
            colsum(dqkv, NT, 3 * D, dbqkv)
            for i in range(3):
                if ctx.has_b[i] and ng[3 + 2 * i]:
                    grads_w[2 * i + 1] = dbqkv[i * D:(i + 1) * D]
        dx = None
        if ng[0]:
            dx = torch.empty(NT, D, device=dev)
            gemm(NT, D, 3 * D, op(dqkv16, 0, 3 * D, True), op(wqkvt16, 0, 3 * D, True), dx, D, residual=dy1)
            dx = dx.view(B, T, D)
        rest = [dwo, dbo, dg1, dbe1, dw1, db1, dw2, db2, dg2, dbe2]
        # small gradients of frozen parameters: accumulated on the side stream too
        for k, g in enumerate(grads_w):
            if g is not None and k % 2 == 1 and _defer_ok(prm[k]):
                _defer_acc(prm[k], g)
                grads_w[k] = None
        for k, g in enumerate(rest):
            if g is not None and _defer_ok(prm[6 + k]):
                _defer_acc(prm[6 + k], g)
                rest[k] = None
            else:
                rest[k] = _mat(g)
        return (dx, None, *grads_w, *rest)


def encoder_layer(x, params, nh, eps, p_attn, p_hid, p_act, training):
    if not training:
        p_attn = p_hid = p_act = 0.0
    seeds = tuple(SEEDS.next() for _ in range(4)) if training else (0, 0, 0, 0)
    cfg = (nh, eps, float(p_attn), float(p_hid), float(p_act), seeds)
    with _fp32_if("enc"):
        if bf16_mode():
            return _EncoderLayer16.apply(x.contiguous(), cfg, *params)
        return _EncoderLayer.apply(x.contiguous(), cfg, *params)


# =====================================================================================
# CTC
# =====================================================================================
class _CTC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, in_lens, tgt_lens, blank):
        _chk(logits, "ctc.logits")
        B, T, C = logits.shape
        S = targets.shape[1]
        dev = logits.device
        ws = torch.empty(int(_lib.load().b2p_ctc_workspace(B, T, S, C)), device=dev)
        nll = torch.empty(B, device=dev)
        loss = torch.empty((), device=dev)
        grad = torch.empty_like(logits)
        _lib.call("b2p_ctc_fwd_bwd", _p(logits), targets.data_ptr(), in_lens.data_ptr(), tgt_lens.data_ptr(), B, T,
                  S, C, blank, _p(nll), _p(loss), _p(grad), _p(ws), _st())
        ctx.save_for_backward(grad)
        ctx.nll = nll
        return loss

    @staticmethod
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        if gout.numel() != 1 or gout.dtype != torch.float32 or gout.device != grad.device:
            return grad * gout, None, None, None, None
        g = torch.empty_like(grad)
        _lib.call("b2p_scale_by_device_scalar", _p(grad), _p(gout.contiguous()), _p(g), grad.numel(), _st())
        return g, None, None, None, None


def unfold_lens(in_lens, kernel: int, stride: int):
    """((in_lens - kernel) / stride).to(torch.int32) (reference src/model/b2p2t_model.py:170-173) in one
    launch (b2p_unfold_lens) for device int64 lengths; any other input takes the reference's expression."""
    if not (in_lens.is_cuda and in_lens.dtype == torch.int64):
        return ((in_lens - kernel) / stride).to(torch.int32)
    x = in_lens.contiguous()
    out = torch.empty(x.shape, device=x.device, dtype=torch.int32)
    _lib.call("b2p_unfold_lens", x.data_ptr(), out.data_ptr(), x.numel(), int(kernel), int(stride), _st())
    return out


def ctc_targets(targets):
    """targets.masked_fill(targets < 1, -100) (reference src/model/w2v_custom_feat_extractor.py:70) in one
    launch (b2p_ctc_targets) for device int64 targets; any other input takes the reference's expression."""
    if not (targets.is_cuda and targets.dtype == torch.int64):
        return targets.masked_fill(targets < 1, -100)
    t = targets.contiguous()
    out = torch.empty_like(t)
    _lib.call("b2p_ctc_targets", t.data_ptr(), out.data_ptr(), t.numel(), _st())
    return out


def loss_seed(loss):
    """The gradient autograd seeds loss.backward() with (ones_like(loss)), one cached device tensor per
    (device, dtype): a captured step then holds no fill launch for it."""
    key = (loss.device, loss.dtype, tuple(loss.shape))
    t = _LOSS_SEEDS.get(key)
    if t is None:
        t = _LOSS_SEEDS[key] = torch.ones(loss.shape, device=loss.device, dtype=loss.dtype)
    return t


_LOSS_SEEDS: dict = {}


def ctc_loss(logits, targets, in_lens, tgt_lens, blank=0):
    """log_softmax(logits) -> nn.CTCLoss(blank, reduction='mean', zero_infinity=True);
    logits (B,T,C) batch-first. targets int64 (B,S); in_lens int32; tgt_lens int64."""
    targets = targets.to(torch.int64).contiguous()
    in_lens = in_lens.to(torch.int32).contiguous()
    tgt_lens = tgt_lens.to(torch.int64).contiguous()
    return _CTC.apply(logits.contiguous(), targets, in_lens, tgt_lens, blank)


def ctc_greedy_wer(logits, targets, blank=0, eos=2, delim=4):
    """Device-side greedy CTC decode + word error rate of a batch (csrc/decode.hip): the train
    evaluator's metric (reference src/train/evaluator.py:69-129) without the host round trip.
    Defaults are the wav2vec2 CTC vocab ids (<pad>=0 blank, </s>=2, '|'=4). Returns
    (wer 0-d tensor, errs (B,) int32, nwords (B,) int32, tokens (B,T) int32, ntok (B,) int32)."""
    _chk(logits, "ctc_greedy_wer.logits")
    B, T, C = logits.shape
    targets = targets.to(torch.int64).contiguous()
    S = targets.shape[1]
    dev = logits.device
    tok = torch.empty(B, T, device=dev, dtype=torch.int32)
    ntok = torch.empty(B, device=dev, dtype=torch.int32)
    errs = torch.empty(B, device=dev, dtype=torch.int32)
    nw = torch.empty(B, device=dev, dtype=torch.int32)
    _lib.call("b2p_ctc_greedy_wer", _p(logits), B, T, C, targets.data_ptr(), S, blank, eos, delim, tok.data_ptr(),
              ntok.data_ptr(), errs.data_ptr(), nw.data_ptr(), _st())
    wer = errs.sum().float() / nw.sum().clamp_min(1).float()
    return wer, errs, nw, tok, ntok


def ctc_prefix_beam(logits, lens=None, beam=100, blank=0, token_min_logp=-5.0, beam_prune_logp=-10.0):
    """LM-free CTC prefix beam search on the device (csrc/beam.hip): the decoding of the reference's
    test evaluator (pyctcdecode via Wav2Vec2ProcessorWithLM, src/train/evaluator.py:189-210) without
    its KenLM model. logits (B, T, C) raw scores; lens (B,) frames per sample (None: T); defaults are
    pyctcdecode's beam width / pruning constants. Returns (tokens (B, T) int32, -1 padded; lengths
    (B,) int32; log probabilities (B,) of the best prefixes)."""
    _chk(logits, "ctc_prefix_beam.logits")
    B, T, C = logits.shape
    dev = logits.device
    lens32 = None if lens is None else lens.to(device=dev, dtype=torch.int32).contiguous()
    ws = torch.empty(int(_lib.load().b2p_ctc_beam_workspace(B, T, beam)), device=dev, dtype=torch.int32)
    tok = torch.empty(B, T, device=dev, dtype=torch.int32)
    n = torch.empty(B, device=dev, dtype=torch.int32)
    score = torch.empty(B, device=dev)
    _lib.call("b2p_ctc_prefix_beam", _p(logits), B, T, C, _p(lens32), beam, blank, float(token_min_logp),
              float(beam_prune_logp), _p(ws), _p(tok), _p(n), _p(score), _st())
    return tok, n, score


_TOKCHARS: dict = {}


def token_char_table(vocab, device):
    """(tok_chars uint8 [C][8], tok_len int32 [C]) device tables of a CTC vocabulary (list of token
    strings, index = id) for ctc_greedy_cer; cached per vocabulary."""
    key = (tuple(vocab), str(device))
    if key not in _TOKCHARS:
        chars = torch.zeros(len(vocab), 8, dtype=torch.uint8)
        lens = torch.zeros(len(vocab), dtype=torch.int32)
        for i, t in enumerate(vocab):
            b = t.encode("utf-8")
            if len(b) > 8:
                raise ValueError(f"token {t!r} longer than 8 bytes")
            chars[i, :len(b)] = torch.tensor(list(b), dtype=torch.uint8)
            lens[i] = len(b)
        _TOKCHARS[key] = (chars.to(device), lens.to(device))
    return _TOKCHARS[key]


def ctc_greedy_cer(logits, targets, vocab, blank=0, eos=2, delim=4):
    """Device-side character error rate of the greedy decode (csrc/decode.hip; reference
    EvaluatorWithW2vLMDecoder.calculate_char_error_rate, src/train/evaluator.py:212-214,231-242).
    Returns (cer 0-d tensor, char_errs (B,) int32, nchars (B,) int32). A row whose decoded string
    overflows the kernel's per-row buffer reports char_errs = -1 and nchars = 0; such rows are left
    out of `cer`, so callers must check char_errs < 0 and score those rows on the host (the
    evaluator does: train/evaluator.py)."""
    _chk(logits, "ctc_greedy_cer.logits")
    B, T, C = logits.shape
    targets = targets.to(torch.int64).contiguous()
    S = targets.shape[1]
    dev = logits.device
    chars, lens = token_char_table(vocab, dev)
    if chars.shape[0] < C:
        raise ValueError(f"vocabulary has {chars.shape[0]} tokens, logits have {C} classes")
    errs = torch.empty(B, device=dev, dtype=torch.int32)
    nch = torch.empty(B, device=dev, dtype=torch.int32)
    _lib.call("b2p_ctc_greedy_cer", _p(logits), B, T, C, targets.data_ptr(), S, blank, eos, delim, chars.data_ptr(),
              lens.data_ptr(), errs.data_ptr(), nch.data_ptr(), _st())
    cer = errs.clamp_min(0).sum().float() / nch.sum().clamp_min(1).float()
    return cer, errs, nch


# =====================================================================================
# Conformer (transformers Wav2Vec2ConformerEncoderLayer, rotary variant) — reference
# src/model/w2v_conformer_custom_feat_extractor.py:62-112
# =====================================================================================
@_gate_aware
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        _chk(x, "layer_norm.x")
        C = x.shape[-1]
        x2 = x.view(-1, C)
        y, mean, rstd = _ln_fwd(x2, g, b, eps)
        ctx.save_for_backward(x2, g, mean, rstd)
        ctx.prm = (g, b)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, g, mean, rstd = ctx.saved_tensors
        dx, dg, db, _ = _ln_bwd(dy.contiguous().view(x2.shape), x2, g, mean, rstd)
        dg, db = _defer_small(ctx.prm, (dg, db))
        return dx.view(dy.shape), dg, db, None


def layer_norm(x, g, b, eps):
    return _LayerNorm.apply(x.contiguous(), g, b, float(eps))


def _dropout_scaled(x, p, seed, scale):
    y = torch.empty_like(x)
    _lib.call("b2p_dropout_scaled", _p(x), _p(y), x.numel(), float(p), seed, float(scale), _st())
    return y


def _drop_cast_colsum(dy, p, seed, scale, want_colsum, lazy=False):
    """(bf16(dropout(dy) * scale), its column sums or None) in one pass over dy (M x N, fp32); lazy:
    the column sums as ColsumParts (for a gradient that goes through _defer_small)."""
    M, N = dy.shape
    y16 = torch.empty(M, N, device=dy.device, dtype=BF16)
    parts = None
    if want_colsum:
        parts = torch.empty(int(_lib.load().b2p_drop_cast_colsum_parts(M)), N, device=dy.device)
    _lib.call("b2p_drop_cast_colsum", _p(dy), _p(y16), _p(parts), M, N, float(p), seed, float(scale), _st())
    if not want_colsum:
        return y16, None
    return y16, (ColsumParts(parts) if lazy else colsum_from_parts(parts, torch.empty(N, device=dy.device)))


def _ln_fwd_x16(x2d, g, b, eps, half, want32=True, want_b16=False):
    """LayerNorm (fp32 y unless want32=False, mean, rstd) plus its 16-bit GEMM operand copy (fp16 when
    half) in one pass; want_b16 adds a bf16 copy (the backward's weight-gradient operand) as a 5th value."""
    rows, cols = x2d.shape
    y = torch.empty_like(x2d) if want32 else None
    y16 = torch.empty(rows, cols, device=x2d.device, dtype=torch.float16 if half else BF16)
    y16b = torch.empty(rows, cols, device=x2d.device, dtype=BF16) if want_b16 else None
    mean = torch.empty(rows, device=x2d.device)
    rstd = torch.empty(rows, device=x2d.device)
    _lib.call("b2p_layernorm_fwd_x16", _p(x2d), _p(g), _p(b), _p(y), _p(y16), int(half), _p(y16b), _p(mean),
              _p(rstd), rows, cols, float(eps), _st())
    if want_b16:
        return y, y16, mean, rstd, y16b
    return y, y16, mean, rstd


# Conformer attention block: LayerNorm + rotary in one launch (B2P_LN_ROT=0: LayerNorm with an fp32
# output, then b2p_rotary16 in the forward and again in the backward)
_LN_ROT = [os.environ.get("B2P_LN_ROT", "1") != "0"]


def ln_rotary16_ok(D, hd) -> bool:
    return D % 256 == 0 and D <= 1024 and hd in (32, 64, 128, 256) and D % hd == 0


def _ln_rotary16(x2d, g, b, eps, T, hd, cos_t, sin_t, half):
    """(h16, h16b, hr16, hr16b, mean, rstd): LayerNorm of x2d and its rotary rotation as 16-bit operands
    (fp16 h16 / hr16 under half, with bf16 copies h16b / hr16b; in bf16 the copies are h16 / hr16)."""
    rows, cols = x2d.shape
    dt = torch.float16 if half else BF16
    dev = x2d.device
    h16 = torch.empty(rows, cols, device=dev, dtype=dt)
    hr16 = torch.empty(rows, cols, device=dev, dtype=dt)
    h16b = torch.empty(rows, cols, device=dev, dtype=BF16) if half else h16
    hr16b = torch.empty(rows, cols, device=dev, dtype=BF16) if half else hr16
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    _lib.call("b2p_layernorm_rotary16", _p(x2d), _p(g), _p(b), _p(mean), _p(rstd), rows, cols, float(eps), T, hd,
              _p(cos_t), _p(sin_t), int(half), _p(h16), _p(h16b) if half else None, _p(hr16),
              _p(hr16b) if half else None, _st())
    return h16, h16b, hr16, hr16b, mean, rstd


def _rotary16(h, cos_t, sin_t, B, T, nh, hd, half):
    out = torch.empty(h.shape, device=h.device, dtype=torch.float16 if half else BF16)
    _lib.call("b2p_rotary16", _p(h), _p(cos_t), _p(sin_t), _p(out), int(half), B, T, nh, hd, h.shape[-1], _st())
    return out


def _w_op16(w, half):
    """(buffer, Operand) of a Linear / pointwise-conv weight [N][K...] as a 16-bit k-contiguous B operand:
    fp16 (the forward_f16 precision; frozen copies cached by _cast_operand) or bf16 (weight16). Keep the
    buffer alive until the GEMM is enqueued."""
    N = w.shape[0]
    K = w.numel() // N
    if half:
        return _cast_operand(op(w, 0, K, True), N, K, True, w.device)
    w16 = weight16(w)
    return w16, op(w16, 0, K, True)


def _act_dropout_cast16(pre, act, p, seed):
    out = torch.empty(pre.shape, device=pre.device, dtype=BF16)
    _lib.call("b2p_act_dropout_cast16", _p(pre), _p(out), pre.numel(), act, float(p), seed, _st())
    return out


_FFN_F16B = [os.environ.get("B2P_FFN_F16B", "1") != "0"]
_BN16 = [os.environ.get("B2P_BN16", "1") != "0"]
_FFN_PRE16 = [os.environ.get("B2P_FFN_PRE16", "1") != "0"]


@_gate_aware
@_prec_follow
class _FFNBlock(torch.autograd.Function):
    """y = x + scale * dropout_h(W2 dropout_a(act(W1 LN(x) + b1)) + b2)   (macaron half-step, scale 0.5)"""

    @staticmethod
    def forward(ctx, x, g, b, w1, b1, w2, b2, cfg):
        ctx.skip = _skip_claim(x)   # LayerDrop skip gradient folded into dx (_SkipSlot)
        act, eps, p_act, p_hid, s_act, s_hid, scale = cfg
        _chk(x, "ffn.x")
        B, T, D = x.shape
        NT, F = B * T, w1.shape[0]
        dev = x.device
        x2 = x.view(NT, D)
        bs = _scaled_bias(b2, scale)
        y = torch.empty(NT, D, device=dev)
        if bf16_mode():
            # 16-bit operands written by their producers (LayerNorm, FFN1 epilogue): no cast passes;
            # fp16 under forward_f16, else bf16. Under forward_f16 the FFN1 epilogue also writes f's
            # bf16 copy, the backward's weight-gradient operand (kept instead of the fp16 one; it was
            # recomputed from pre, a 195 MB pass per FFN at Conformer-large bs=32)
            half = _state.fwd16
            # the pre-activation is read only by the backward's act' (the GEMM epilogue's aux16 operand):
            # stored in bf16 (B2P_FFN_PRE16=0: fp32), half the bytes written and read back
            pre16 = _FFN_PRE16[0] and (not half or _FFN_F16B[0])
            pre = torch.empty(NT, F, device=dev, dtype=BF16 if pre16 else torch.float32)
            if half:   # h kept only as the bf16 weight-gradient operand of the backward (no fp32 copy)
                _, h16, mean, rstd, h = _ln_fwd_x16(x2, g, b, eps, half, want32=False, want_b16=True)
            else:
                _, h16, mean, rstd = _ln_fwd_x16(x2, g, b, eps, half, want32=False)
                h = h16
            f = torch.empty(NT, F, device=dev, dtype=torch.float16 if half else BF16)
            fb = torch.empty(NT, F, device=dev, dtype=BF16) if half and _FFN_F16B[0] else None
            w1b, w1op = _w_op16(w1, half)
            gemm(NT, F, D, op(h16, 0, D, True), w1op, None, F, bias=b1, pre_out=None if pre16 else pre,
                 pre16=pre if pre16 else None, act=act, drop_p=p_act, seed=s_act, C16=f, c16_fp16=half, C16b=fb)
            del h16, w1b
            w2b, w2op = _w_op16(w2, half)
            gemm(NT, D, F, op(f, 0, F, True), w2op, y, D, alpha=scale, bias=bs, drop_p=p_hid, seed=s_hid,
                 residual=x2)
            del w2b
            if fb is not None:
                f = fb
        else:
            pre = torch.empty(NT, F, device=dev)
            h, mean, rstd = _ln_fwd(x2, g, b, eps)
            f = torch.empty(NT, F, device=dev)
            gemm(NT, F, D, op(h, 0, D, True), op(w1, 0, D, True), f, F, bias=b1, pre_out=pre, act=act, drop_p=p_act,
                 seed=s_act)
            gemm(NT, D, F, op(f, 0, F, True), op(w2, 0, F, True), y, D, alpha=scale, bias=bs, drop_p=p_hid,
                 seed=s_hid, residual=x2)
        ctx.save_for_backward(x2, h, mean, rstd, pre, f, g, w1, w2)
        ctx.cfg = cfg
        ctx.shape = (B, T, D)
        ctx.has_b = (b1 is not None, b2 is not None)
        ctx.prm = (g, b, w1, b1, w2, b2)
        return y.view(B, T, D)

    @staticmethod
    def backward(ctx, dy):
        x2, h, mean, rstd, pre, f, g, w1, w2 = ctx.saved_tensors
        act, eps, p_act, p_hid, s_act, s_hid, scale = ctx.cfg
        NT, D = x2.shape
        F = w1.shape[0]
        dev = x2.device
        ng = ctx.needs_input_grad
        dy = dy.contiguous().view(NT, D)
        if _bwd16_path() or h.dtype != torch.float32:
            return _FFNBlock._backward16(ctx, dy, x2, h, mean, rstd, pre, f, g, w1, w2)
        dz = _dropout_scaled(dy, p_hid, s_hid, scale)
        dw2 = db2 = dw1 = db1 = None
        if ng[5]:
            dw2 = torch.empty_like(w2)
            mm_tn(dz, f, dw2)
        if ctx.has_b[1] and ng[6]:
            db2 = torch.empty(D, device=dev)
            colsum(dz, NT, D, db2)
        dpre = torch.empty(NT, F, device=dev)
        gemm(NT, F, D, op(dz, 0, D, True), op(w2, 0, F, False), dpre, F, drop_p=p_act, seed=s_act, act_bwd=act,
             aux=pre)
        if ng[3]:
            dw1 = torch.empty_like(w1)
            mm_tn(dpre, h, dw1)
        if ctx.has_b[0] and ng[4]:
            db1 = torch.empty(F, device=dev)
            colsum(dpre, NT, F, db1)
        dh = torch.empty(NT, D, device=dev)
        mm_nn(dpre, w1, dh)
        dx, dg, db, _, _ = _ln_bwd(dh, x2, g, mean, rstd, True, dx_accum=dy, dx_accum2=_skip_take(ctx.skip),
                                   lazy=(ctx.prm[0], ctx.prm[1], None))
        return (dx.view(ctx.shape), *_defer_small(ctx.prm, (dg, db, dw1, db1, dw2, db2)), None)

    @staticmethod
    def _backward16(ctx, dy, x2, h, mean, rstd, pre, f, g, w1, w2):
        """bf16-operand backward (same math): the output dropout, its bf16 copy and the FFN2 bias
        gradient in one pass over dy; f, h cast once; dpre produced in bf16 by the backward-data
        GEMM with the FFN1 bias gradient as fused column sums; weight gradients of frozen
        parameters deferred (accumulated into .grad by the GEMM)."""
        act, eps, p_act, p_hid, s_act, s_hid, scale = ctx.cfg
        NT, D = x2.shape
        F = w1.shape[0]
        dev = x2.device
        ng = ctx.needs_input_grad
        dz16, db2 = _drop_cast_colsum(dy, p_hid, s_hid, scale, ctx.has_b[1] and ng[6], lazy=True)
        db1 = None
        f16 = f if f.dtype == BF16 else _act_dropout_cast16(pre, act, p_act, s_act)
        dw2 = _wgrad16(w2, ng[5], dz16, D, f16, F, NT)
        del f16
        dpre16 = torch.empty(NT, F, device=dev, dtype=BF16)
        parts = colsum_parts_buf(NT, F, dev) if (ctx.has_b[0] and ng[4]) else None
        gemm(NT, F, D, op(dz16, 0, D, True), op(weight16t(w2), 0, D, True), None, F, drop_p=p_act, seed=s_act,
             act_bwd=act, aux=None if pre.dtype == BF16 else pre, aux16=pre if pre.dtype == BF16 else None,
             C16=dpre16, colsum_part=parts)
        if parts is not None:
            db1 = ColsumParts(parts)   # finished by _defer_small (side-stream launch or materialised)
        dw1 = _wgrad16(w1, ng[3], dpre16, F, h if h.dtype == BF16 else cast16(h), D, NT)
        dh = torch.empty(NT, D, device=dev)
        gemm(NT, D, F, op(dpre16, 0, F, True), op(weight16t(w1), 0, F, True), dh, D)
        dx, dg, db, _, _ = _ln_bwd(dh, x2, g, mean, rstd, True, dx_accum=dy, dx_accum2=_skip_take(ctx.skip),
                                   lazy=(ctx.prm[0], ctx.prm[1], None))
        return (dx.view(ctx.shape), *_defer_small(ctx.prm, (dg, db, dw1, db1, dw2, db2)), None)


def _wgrad16(w, need, dy16, M, x16, N, NT, ldy=None, ldx=None, dy_off=0):
    """Weight gradient dW[M][N] = dy16[:, off:off+M]^T x16 (bf16 operands, K = NT tokens): deferred
    onto the side stream and accumulated into w.grad (beta = 1) for a frozen parameter, else
    returned. None when not needed."""
    if not need:
        return None
    ldy, ldx = ldy or M, ldx or N
    if _defer_ok(w):
        _defer_wspec((w,), M, N, NT, dy16, dy_off, ldy, x16, ldx)
        return None
    gw = torch.empty_like(w)
    gemm(M, N, NT, op(dy16, dy_off, ldy, False), op(x16, 0, ldx, False), gw, N)
    return gw


_ROT = {}


def rotary_tables(T, D, base, device):
    """TF conf Wav2Vec2ConformerRotaryPositionalEmbedding: inv_freq = base^(-arange(0,D,2)/D),
    emb = cat(t*inv_freq, t*inv_freq) -> (cos, sin) of shape (T, D). Cached per (T, D, base)."""
    key = (T, D, base, str(device))
    if key not in _ROT:
        # first use inside a graph capture (no host-to-device copy allowed): build the table on the
        # device, as the reference's own module does (TF conf builds it on hidden_states.device)
        on = torch.device(device) if capturing() else torch.device("cpu")
        inv_freq = 1.0 / (base ** (torch.arange(0, D, 2, dtype=torch.int64, device=on).float() / D))
        t = torch.arange(T, device=on).type_as(inv_freq)
        freqs = torch.einsum("i,j->ij", t, inv_freq)
        emb = torch.cat((freqs, freqs), dim=-1)
        _ROT[key] = (emb.cos().contiguous().to(device), emb.sin().contiguous().to(device))
    return _ROT[key]


@_gate_aware
@_prec_follow
class _ConformerAttnBlock(torch.autograd.Function):
    """y = x + dropout(linear_out(Attn(q=k=rotary(LN x), v=LN x)))  (TF conf Wav2Vec2ConformerSelfAttention)"""

    @staticmethod
    def forward(ctx, x, g, b, wq, bq, wk, bk, wv, bv, wo, bo, cos_t, sin_t, cfg):
        ctx.skip = _skip_claim(x)   # LayerDrop skip gradient folded into dx (_SkipSlot)
        nh, eps, p_attn, p_out, seeds = cfg
        _chk(x, "conformer_attn.x")
        B, T, D = x.shape
        NT, hd = B * T, D // nh
        dev = x.device
        x2 = x.view(NT, D)
        # bf16 mode, head 64, T' <= 256: fused attention (csrc/attn16.hip, scores stay on-chip); the
        # QKV GEMMs then write only the bf16 operand, and the saved slots hold qkv16 / lse2 / dropout
        # keep bits / O16
        ctx.fused = bf16_mode() and attn16_ok(T, hd)
        # fused: the 16-bit attention operand (fp16 under ATTN_F16: the backward recomputes from it)
        qkv = torch.empty(NT, 3 * D, device=dev, dtype=(torch.float16 if ATTN_F16 else BF16) if ctx.fused
                          else torch.float32)
        f16a = ctx.fused and ATTN_F16
        if bf16_mode():
            # the Q/K/V operands come straight from their producers as 16-bit copies (LayerNorm, rotary):
            # fp16 under forward_f16, else bf16; the fp32 rotated copy is never stored
            half = _state.fwd16
            hr16b = None
            if cos_t is not None and _LN_ROT[0] and _bwd16_path() and ln_rotary16_ok(D, hd):
                # LayerNorm + rotary in one pass, 16-bit outputs only (no fp32 LN output, no rotary
                # launches): the backward keeps the bf16 rotated copy for the Q/K weight gradients
                h16, h16b, hr16, hr16b, mean, rstd = _ln_rotary16(x2, g, b, eps, T, hd, cos_t, sin_t, half)
                h = None
            elif half:   # fp16 operand for the forward GEMMs, bf16 copy for the V weight gradient
                h, h16, mean, rstd, h16b = _ln_fwd_x16(x2, g, b, eps, half, want_b16=True)
            else:
                h, h16, mean, rstd = _ln_fwd_x16(x2, g, b, eps, half)
                h16b = h16
            if h is not None:
                hr16 = _rotary16(h, cos_t, sin_t, B, T, nh, hd, half) if cos_t is not None else h16
            hr = None
            for i, (w, bb, src) in enumerate(((wq, bq, hr16), (wk, bk, hr16), (wv, bv, h16))):
                wbuf, wop = _w_op16(w, half)
                if f16a:
                    gemm(NT, D, D, op(src, 0, D, True), wop, None, 3 * D, c_off=i * D, bias=bb, C16=qkv,
                         c16_fp16=True)
                elif ctx.fused:
                    gemm(NT, D, D, op(src, 0, D, True), wop, None, 3 * D, c_off=i * D, bias=bb, C16=qkv)
                else:
                    gemm(NT, D, D, op(src, 0, D, True), wop, qkv, 3 * D, c_off=i * D, bias=bb)
                del wbuf
            del h16, hr16
        else:
            h16b = hr16b = None
            h, mean, rstd = _ln_fwd(x2, g, b, eps)
            if cos_t is not None:
                hr = torch.empty_like(h)
                _lib.call("b2p_rotary", _p(h), _p(cos_t), _p(sin_t), _p(hr), B, T, nh, hd, D, 0, _st())
            else:
                hr = h
            for i, (w, bb, src) in enumerate(((wq, bq, hr), (wk, bk, hr), (wv, bv, h))):
                gemm(NT, D, D, op(src, 0, D, True), op(w, 0, D, True), qkv, 3 * D, c_off=i * D, bias=bb)
        y = torch.empty(NT, D, device=dev)
        if f16a:
            Oh, O, P, Pd = _attn16_fwd_f16(qkv, B, T, nh, hd, p_attn, seeds[0])
            wbuf, wop = _w_op16(wo, True)
            gemm(NT, D, D, op(Oh, 0, D, True), wop, y, D, bias=bo, drop_p=p_out, seed=seeds[1], residual=x2)
            del Oh, wbuf
        elif ctx.fused:
            O, P, Pd = _attn16_fwd(qkv, B, T, nh, hd, p_attn, seeds[0], want_mask=True)
            gemm(NT, D, D, op(O, 0, D, True), op(weight16(wo), 0, D, True), y, D, bias=bo, drop_p=p_out,
                 seed=seeds[1], residual=x2)
        else:
            P, Pd, O = _attn_core_fwd(qkv, B, T, nh, hd, p_attn, seeds[0])
            gemm(NT, D, D, op(O, 0, D, True), op(wo, 0, D, True), y, D, bias=bo, drop_p=p_out, seed=seeds[1],
                 residual=x2)
        ctx.save_for_backward(x2, h, hr if (cos_t is not None and hr is not None) else None, mean, rstd, qkv, P, Pd,
                              O, g, wq, wk, wv, wo, cos_t, sin_t, h16b, hr16b)
        ctx.cfg = cfg
        ctx.shape = (B, T, D)
        ctx.has_b = [t is not None for t in (bq, bk, bv, bo)]
        ctx.prm = (g, b, wq, bq, wk, bk, wv, bv, wo, bo)
        return y.view(B, T, D)

    @staticmethod
    def backward(ctx, dy):
        x2, h, hr, mean, rstd, qkv, P, Pd, O, g, wq, wk, wv, wo, cos_t, sin_t, h16b, hr16b = ctx.saved_tensors
        ctx.h16b = h16b
        ctx.hr16b = hr16b
        nh, eps, p_attn, p_out, seeds = ctx.cfg
        B, T, D = ctx.shape
        NT, hd = B * T, D // nh
        dev = x2.device
        ng = ctx.needs_input_grad
        hr_ = h if hr is None else hr
        dy = dy.contiguous().view(NT, D)
        if _bwd16_path() or ctx.fused:
            return _ConformerAttnBlock._backward16(ctx, dy, x2, h, hr, mean, rstd, qkv, P, Pd, O, g, wq, wk, wv,
                                                   wo, cos_t, sin_t)
        dz = _dropout_scaled(dy, p_out, seeds[1], 1.0)
        dwo = dbo = None
        if ng[9]:
            dwo = torch.empty_like(wo)
            mm_tn(dz, O, dwo)
        if ctx.has_b[3] and ng[10]:
            dbo = torch.empty(D, device=dev)
            colsum(dz, NT, D, dbo)
        dO = torch.empty(NT, D, device=dev)
        mm_nn(dz, wo, dO)
        dqkv = _attn_core_bwd(qkv, P, Pd, dO, B, T, nh, hd, p_attn, seeds[0])
        grads = []
        for i, (w, src) in enumerate(((wq, hr_), (wk, hr_), (wv, h))):
            gw = gb = None
            if ng[3 + 2 * i]:
                gw = torch.empty_like(w)
                gemm(D, D, NT, op(dqkv, i * D, 3 * D, False), op(src, 0, D, False), gw, D)
            if ctx.has_b[i] and ng[4 + 2 * i]:
                gb = torch.empty(D, device=dev)
                colsum(_view_off(dqkv, i * D), NT, D, gb, ld=3 * D)
            grads += [gw, gb]
        # dh = rotary^T(dQ Wq + dK Wk) + dV Wv
        dh = torch.empty(NT, D, device=dev)
        if cos_t is not None:
            dhr = torch.empty(NT, D, device=dev)
            gemm(NT, D, D, op(dqkv, 0, 3 * D, True), op(wq, 0, D, False), dhr, D)
            gemm(NT, D, D, op(dqkv, D, 3 * D, True), op(wk, 0, D, False), dhr, D, beta=1.0)
            _lib.call("b2p_rotary", _p(dhr), _p(cos_t), _p(sin_t), _p(dh), B, T, nh, hd, D, 1, _st())
            gemm(NT, D, D, op(dqkv, 2 * D, 3 * D, True), op(wv, 0, D, False), dh, D, beta=1.0)
        else:
            for i, w in enumerate((wq, wk, wv)):
                gemm(NT, D, D, op(dqkv, i * D, 3 * D, True), op(w, 0, D, False), dh, D, beta=0.0 if i == 0 else 1.0)
        dx, dg, db, _, _ = _ln_bwd(dh, x2, g, mean, rstd, True, dx_accum=dy, dx_accum2=_skip_take(ctx.skip),
                                   lazy=(ctx.prm[0], ctx.prm[1], None))
        return (dx.view(B, T, D), *_defer_small(ctx.prm, (dg, db, *grads, dwo, dbo)), None, None, None)

    @staticmethod
    def _backward16(ctx, dy, x2, h, hr, mean, rstd, qkv, P, Pd, O, g, wq, wk, wv, wo, cos_t, sin_t):
        """bf16-operand backward (same math): every GEMM operand cast once, Q/K (and V without
        rotary) input gradients as one GEMM over the concatenated transposed weights, frozen
        weight gradients deferred."""
        nh, eps, p_attn, p_out, seeds = ctx.cfg
        B, T, D = ctx.shape
        NT, hd = B * T, D // nh
        dev = x2.device
        ng = ctx.needs_input_grad
        dz16, dbo = _drop_cast_colsum(dy, p_out, seeds[1], 1.0, ctx.has_b[3] and ng[10], lazy=True)
        dwo = _wgrad16(wo, ng[9], dz16, D, O if ctx.fused else cast16(O), D, NT)
        if ctx.fused:
            # qkv / P / Pd / O hold qkv16, lse2, the dropout keep bits and O16 (forward)
            dO16 = torch.empty(NT, D, device=dev, dtype=BF16)
            gemm(NT, D, D, op(dz16, 0, D, True), op(weight16t(wo), 0, D, True), None, D, C16=dO16)
            dqkv, dqkv16 = _attn16_bwd(qkv, dO16, P, B, T, nh, hd, p_attn, seeds[0], mask=Pd)
            del dO16
        else:
            dO = torch.empty(NT, D, device=dev)
            gemm(NT, D, D, op(dz16, 0, D, True), op(weight16t(wo), 0, D, True), dO, D)
            dqkv = _attn_core_bwd(qkv, P, Pd, dO, B, T, nh, hd, p_attn, seeds[0])
            del dO
            dqkv16 = cast16(dqkv)
        h16 = ctx.h16b if ctx.h16b is not None else cast16(h)
        if cos_t is None:
            hr16 = h16
        elif ctx.hr16b is not None:   # LayerNorm + rotary forward: its bf16 rotated copy
            hr16 = ctx.hr16b
        elif hr is None:   # the forward kept no fp32 rotated copy: rotate h again, into bf16
            hr16 = _rotary16(h, cos_t, sin_t, B, T, nh, hd, False)
        else:
            hr16 = cast16(hr)
        grads = []
        need_b = [ctx.has_b[i] and ng[4 + 2 * i] for i in range(3)]
        dbqkv = None
        b_side = all(need_b) and _defer_bias_rows((ctx.prm[3], ctx.prm[5], ctx.prm[7]), dqkv, NT, 3 * D)
        if all(need_b) and not b_side:   # the three bias gradients as one column reduction over dqkv
            dbqkv = torch.empty(3 * D, device=dev)
            colsum(dqkv, NT, 3 * D, dbqkv)
        for i, (w, src16) in enumerate(((wq, hr16), (wk, hr16), (wv, h16))):
            gb = None
            if b_side:
                pass
            elif dbqkv is not None:
                gb = dbqkv[i * D:(i + 1) * D]
            elif need_b[i]:
                gb = torch.empty(D, device=dev)
                colsum(_view_off(dqkv, i * D), NT, D, gb, ld=3 * D)
            grads += [_wgrad16(w, ng[3 + 2 * i], dqkv16, D, src16, D, NT, ldy=3 * D, dy_off=i * D), gb]
        del dqkv
        dh = torch.empty(NT, D, device=dev)
        if cos_t is not None:
            # dh = rotary^T([dQ dK] [Wq; Wk]) + dV Wv
            dhr = torch.empty(NT, D, device=dev)
            gemm(NT, D, 2 * D, op(dqkv16, 0, 3 * D, True), op(weight16t(wq, wk), 0, 2 * D, True), dhr, D)
            _lib.call("b2p_rotary", _p(dhr), _p(cos_t), _p(sin_t), _p(dh), B, T, nh, hd, D, 1, _st())
            gemm(NT, D, D, op(dqkv16, 2 * D, 3 * D, True), op(weight16t(wv), 0, D, True), dh, D, beta=1.0)
        else:
            gemm(NT, D, 3 * D, op(dqkv16, 0, 3 * D, True), op(weight16t(wq, wk, wv), 0, 3 * D, True), dh, D)
        dx, dg, db, _, _ = _ln_bwd(dh, x2, g, mean, rstd, True, dx_accum=dy, dx_accum2=_skip_take(ctx.skip),
                                   lazy=(ctx.prm[0], ctx.prm[1], None))
        return (dx.view(B, T, D), *_defer_small(ctx.prm, (dg, db, *grads, dwo, dbo)), None, None, None)


# ------------------------------------------------------------------ synchronised BatchNorm
def _bn_fwd_sync(c, gamma, beta, run_mean, run_var, y, pre, mean, rstd, M, C, eps, momentum, act, ws, group, y16=None,
                 half=False, y16b=None):
    """Training BatchNorm over the rows of every data-parallel rank: the
    per-channel sum and the sum of squared deviations from the global mean are all-reduced
    (2 x C floats per conv module); running statistics use the global count, like torch SyncBN."""
    import torch.distributed as dist
    count = M * dist.get_world_size(group)
    _lib.call("b2p_batchnorm_stats", _p(c), None, _p(mean), M, C, _p(ws), _st())
    collective(lambda: dist.all_reduce(mean, group=group))
    _lib.call("b2p_batchnorm_finalize", _p(mean), None, None, None, None, C, count, float(eps), float(momentum), 0,
              _st())
    sq = torch.empty(C, device=c.device)
    _lib.call("b2p_batchnorm_stats", _p(c), _p(mean), _p(sq), M, C, _p(ws), _st())
    collective(lambda: dist.all_reduce(sq, group=group))
    _lib.call("b2p_batchnorm_finalize", _p(mean), _p(sq), _p(rstd), _p(run_mean), _p(run_var), C, count, float(eps),
              float(momentum), 1, _st())
    if y16 is not None:   # 16-bit operand outputs (y may be None)
        _lib.call("b2p_batchnorm_apply16", _p(c), _p(mean), _p(rstd), _p(gamma), _p(beta), _p(y), _p(y16), int(half),
                  _p(y16b), _p(pre), M, C, act, _st())
    else:
        _lib.call("b2p_batchnorm_apply", _p(c), _p(mean), _p(rstd), _p(gamma), _p(beta), _p(y), _p(pre), M, C, act,
                  _st())


def _bn_bwd_sync(dy, pre, c, mean, rstd, gamma, dx, dgamma, dbeta, M, C, act, ws, group):
    """Backward of _bn_fwd_sync: the per-channel sums of g and g * xhat are all-reduced for the input
    gradient (one 2C all-reduce); dgamma / dbeta stay this rank's sums (the gradient all-reduce
    averages them like every other parameter)."""
    import torch.distributed as dist
    count = M * dist.get_world_size(group)
    g = torch.empty(M, C, device=c.device)
    _lib.call("b2p_batchnorm_bwd_sums", _p(dy), _p(pre), _p(c), _p(mean), _p(rstd), _p(g), _p(dbeta), _p(dgamma), M,
              C, act, _p(ws), _st())
    sums = torch.cat([dbeta, dgamma])
    collective(lambda: dist.all_reduce(sums, group=group))
    _lib.call("b2p_batchnorm_bwd_dx", _p(g), _p(c), _p(mean), _p(rstd), _p(gamma), _p(sums), _p(sums, C), _p(dx), M, C,
              count, _st())


@contextlib.contextmanager
def sync_batchnorm(group):
    """Training-mode BatchNorm inside uses statistics synchronised over `group` (None: local)."""
    old = _state.sync_bn
    _state.sync_bn = group
    try:
        yield
    finally:
        _state.sync_bn = old


@_gate_aware
@_prec_follow
class _ConvModule(torch.autograd.Function):
    """y = x + dropout(pw2(act(BN(dwconv(GLU(pw1(LN x)))))))   (TF conf Wav2Vec2ConformerConvolutionModule)"""

    @staticmethod
    def forward(ctx, x, g, b, w_pw1, w_dw, bn_g, bn_b, w_pw2, bn_rm, bn_rv, cfg):
        act, eps, bn_eps, momentum, p, seed, training, nbt = cfg
        _chk(x, "conv_module.x")
        B, T, D = x.shape
        NT = B * T
        K = w_dw.shape[-1]
        dev = x.device
        x2 = x.view(NT, D)
        a = torch.empty(NT, 2 * D, device=dev)
        if bf16_mode():   # the pointwise-conv operand written by the LayerNorm (fp16 under forward_f16)
            half = _state.fwd16
            if half:      # h kept only as the bf16 operand of the pw1 weight gradient
                _, h16, mean, rstd, h = _ln_fwd_x16(x2, g, b, eps, half, want32=False, want_b16=True)
            else:
                _, h16, mean, rstd = _ln_fwd_x16(x2, g, b, eps, half, want32=False)
                h = h16
            wbuf, wop = _w_op16(w_pw1, half)
            gemm(NT, 2 * D, D, op(h16, 0, D, True), wop, a, 2 * D)
            del h16, wbuf
        else:
            h, mean, rstd = _ln_fwd(x2, g, b, eps)
            gemm(NT, 2 * D, D, op(h, 0, D, True), op(w_pw1, 0, D, True), a, 2 * D)
        u = torch.empty(NT, D, device=dev)
        _lib.call("b2p_glu_fwd", _p(a), _p(u), NT, D, _st())
        c = torch.empty(NT, D, device=dev)
        _lib.call("b2p_dwconv_fwd", _p(u), _p(w_dw), _p(c), B, T, D, K, _st())
        ws = torch.empty(int(_lib.load().b2p_batchnorm_workspace(NT, D)), device=dev)
        sync = None
        # bf16 training step: the BatchNorm + activation writes only the 16-bit operands of pointwise conv 2
        # (its forward GEMM: fp16 under forward_f16; its weight gradient: bf16), no fp32 output and no cast
        # passes (B2P_BN16=0: fp32 output, operands cast from it)
        o16 = training and _BN16[0] and bf16_mode() and _bwd16_path() and D % 4 == 0
        half = o16 and _state.fwd16
        s = None if o16 else torch.empty(NT, D, device=dev)
        s16 = torch.empty(NT, D, device=dev, dtype=torch.float16 if half else BF16) if o16 else None
        s16b = torch.empty(NT, D, device=dev, dtype=BF16) if half else None
        if training:
            pre = torch.empty(NT, D, device=dev)
            bm = torch.empty(D, device=dev)
            br = torch.empty(D, device=dev)
            sync = _state.sync_bn
            if nbt is not None:
                _lib.call("b2p_batchnorm_count_next", _p(nbt))
            if sync is not None:
                _bn_fwd_sync(c, bn_g, bn_b, bn_rm, bn_rv, s, pre, bm, br, NT, D, bn_eps, momentum, act, ws, sync,
                             y16=s16, half=half, y16b=s16b)
            elif o16:
                _lib.call("b2p_batchnorm_fwd16", _p(c), _p(bn_g), _p(bn_b), _p(bn_rm), _p(bn_rv), None, _p(s16),
                          int(half), _p(s16b), _p(pre), _p(bm), _p(br), NT, D, float(bn_eps), float(momentum), act,
                          _p(ws), _st())
            else:
                _lib.call("b2p_batchnorm_fwd", _p(c), _p(bn_g), _p(bn_b), _p(bn_rm), _p(bn_rv), _p(s), _p(pre),
                          _p(bm), _p(br), NT, D, float(bn_eps), float(momentum), act, _p(ws), _st())
        else:
            pre = bm = br = None
            _lib.call("b2p_batchnorm_eval", _p(c), _p(bn_g), _p(bn_b), _p(bn_rm), _p(bn_rv), _p(s), NT, D,
                      float(bn_eps), act, _p(ws), _st())
        y = torch.empty(NT, D, device=dev)
        if o16:
            wbuf, wop = _w_op16(w_pw2, half)
            gemm(NT, D, D, op(s16, 0, D, True), wop, y, D, drop_p=p, seed=seed, residual=x2)
            del wbuf
            s = s16b if half else s16   # the bf16 weight-gradient operand is what the backward keeps
        else:
            gemm(NT, D, D, op(s, 0, D, True), op(w_pw2, 0, D, True), y, D, drop_p=p, seed=seed, residual=x2)
        ctx.save_for_backward(x2, h, mean, rstd, a, u, c, pre, bm, br, s, g, w_pw1, w_dw, bn_g, w_pw2)
        ctx.cfg = cfg
        ctx.shape = (B, T, D, K)
        ctx.sync = sync
        ctx.prm = (g, b, w_pw1, w_dw, bn_g, bn_b, w_pw2)
        return y.view(B, T, D)

    @staticmethod
    def backward(ctx, dy):
        x2, h, mean, rstd, a, u, c, pre, bm, br, s, g, w_pw1, w_dw, bn_g, w_pw2 = ctx.saved_tensors
        act, eps, bn_eps, momentum, p, seed, training, _ = ctx.cfg
        if not training:
            raise RuntimeError("conv module backward in eval mode (running BN statistics) is not supported")
        B, T, D, K = ctx.shape
        NT = B * T
        dev = x2.device
        ng = ctx.needs_input_grad
        dy = dy.contiguous().view(NT, D)
        b16 = _bwd16_path() or h.dtype != torch.float32   # bf16 operands: each cast once, frozen wgrads deferred
        ds = torch.empty(NT, D, device=dev)
        if b16:
            do16, _ = _drop_cast_colsum(dy, p, seed, 1.0, False)
            dpw2 = _wgrad16(w_pw2, ng[7], do16, D, s if s.dtype == BF16 else cast16(s), D, NT)
            gemm(NT, D, D, op(do16, 0, D, True), op(weight16t(w_pw2), 0, D, True), ds, D)
            del do16
        else:
            do = _dropout_scaled(dy, p, seed, 1.0)
            dpw2 = None
            if ng[7]:
                dpw2 = torch.empty_like(w_pw2)
                mm_tn(do, s, dpw2.view(D, D))
            mm_nn(do, w_pw2.view(D, D), ds)
        dc = torch.empty(NT, D, device=dev)
        dbn_g = torch.empty(D, device=dev)
        dbn_b = torch.empty(D, device=dev)
        ws = torch.empty(int(_lib.load().b2p_batchnorm_workspace(NT, D)), device=dev)
        if ctx.sync is not None:
            _bn_bwd_sync(ds, pre, c, bm, br, bn_g, dc, dbn_g, dbn_b, NT, D, act, ws, ctx.sync)
        else:
            _lib.call("b2p_batchnorm_bwd", _p(ds), _p(pre), _p(c), _p(bm), _p(br), _p(bn_g), _p(dc), _p(dbn_g),
                      _p(dbn_b), NT, D, act, _p(ws), _st())
        du = torch.empty(NT, D, device=dev)
        ddw = None
        if ng[4]:
            if _defer_ok(w_dw) and _LAZY_COLSUM:
                _defer_dwconv_wgrad(w_dw, u, dc, B, T, D, K)   # frozen taps: their three launches on the side stream
            else:
                ddw = torch.empty_like(w_dw)
        wsd = torch.empty(int(_lib.load().b2p_dwconv_bwd_workspace(B, T, D, K)), device=dev)
        _lib.call("b2p_dwconv_bwd", _p(u), _p(w_dw), _p(dc), _p(du), _p(ddw), B, T, D, K, _p(wsd), _st())
        dh = torch.empty(NT, D, device=dev)
        if b16:   # the GLU backward writes the bf16 GEMM operand directly
            da16 = torch.empty(NT, 2 * D, device=dev, dtype=BF16)
            _lib.call("b2p_glu_bwd16", _p(a), _p(du), _p(da16), NT, D, _st())
            dpw1 = _wgrad16(w_pw1, ng[3], da16, 2 * D, h if h.dtype == BF16 else cast16(h), D, NT)
            gemm(NT, D, 2 * D, op(da16, 0, 2 * D, True), op(weight16t(w_pw1), 0, 2 * D, True), dh, D)
        else:
            da = torch.empty(NT, 2 * D, device=dev)
            _lib.call("b2p_glu_bwd", _p(a), _p(du), _p(da), NT, D, _st())
            dpw1 = None
            if ng[3]:
                dpw1 = torch.empty_like(w_pw1)
                mm_tn(da, h, dpw1.view(2 * D, D))
            mm_nn(da, w_pw1.view(2 * D, D), dh)
        dx, dg, db, _, _ = _ln_bwd(dh, x2, g, mean, rstd, True, dx_accum=dy, lazy=(ctx.prm[0], ctx.prm[1], None))
        return (dx.view(B, T, D), *_defer_small(ctx.prm, (dg, db, dpw1, ddw, dbn_g, dbn_b, dpw2)), None, None, None)


def conformer_ffn(x, ln, w1, b1, w2, b2, act, p_act, p_hid, training, scale=0.5):
    if not training:
        p_act = p_hid = 0.0
    cfg = (act, float(ln.eps), float(p_act), float(p_hid), SEEDS.next() if p_act > 0 else 0,
           SEEDS.next() if p_hid > 0 else 0, float(scale))
    with _fp32_if("ffn"):
        return _FFNBlock.apply(x.contiguous(), ln.weight, ln.bias, w1, b1, w2, b2, cfg)


def conformer_attention(x, ln, q, k, v, o, nh, rotary, p_attn, p_out, training):
    if not training:
        p_attn = p_out = 0.0
    B, T, D = x.shape
    cos_t = sin_t = None
    if rotary is not None:
        cos_t, sin_t = rotary_tables(T, D // nh, rotary, x.device)
    seeds = (SEEDS.next() if p_attn > 0 else 0, SEEDS.next() if p_out > 0 else 0)
    cfg = (nh, float(ln.eps), float(p_attn), float(p_out), seeds)
    with _fp32_if("attn"):
        return _ConformerAttnBlock.apply(x.contiguous(), ln.weight, ln.bias, q.weight, q.bias, k.weight, k.bias,
                                         v.weight, v.bias, o.weight, o.bias, cos_t, sin_t, cfg)


def conformer_conv_module(x, cm, act, p, training):
    bn = cm.batch_norm
    if not training:
        p = 0.0
    # num_batches_tracked += 1 (torch _BatchNorm.forward in training) happens on the device, inside the
    # statistics launch and under the LayerDrop gate (b2p_batchnorm_count_next)
    nbt = bn.num_batches_tracked if training and bn.track_running_stats else None
    cfg = (act, float(cm.layer_norm.eps), float(bn.eps), float(bn.momentum if bn.momentum is not None else 0.1),
           float(p), SEEDS.next() if p > 0 else 0, bool(training), nbt)
    with _fp32_if("conv"):
        return _ConvModule.apply(x.contiguous(), cm.layer_norm.weight, cm.layer_norm.bias, cm.pointwise_conv1.weight,
                                 cm.depthwise_conv.weight, bn.weight, bn.bias, cm.pointwise_conv2.weight,
                                 bn.running_mean, bn.running_var, cfg)
