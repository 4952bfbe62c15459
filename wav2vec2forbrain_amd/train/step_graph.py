"""StepGraph: one whole training step (forward, CTC, backward, the side-stream frozen-parameter
gradients, Adam) captured once as a HIP graph and replayed per step.

The reference's step (src/train/train_loop.py:41-84) is ~560 kernel launches issued from Python;
on MI355X the host needs about as long to issue them as the GPU needs to run them, so an eager
step idles the GPU between launches. Replaying the captured graph issues the whole step with one
call. What stays live across replays:
  * dropout masks: every dropout kernel adds a device step counter (b2p_set_seed_epoch) to its
    host-drawn seed; the counter's increment is the graph's first node, so each replay draws new
    masks (the per-call seeds drawn at capture time only fix the call sites apart);
  * Adam: HipAdam.make_capturable keeps lr and the step count on the device
    (b2p_adam_multi_dev); prepare_replay() refreshes lr from the param groups (schedulers),
    after_replay() advances the host step counters;
  * inputs: the step reads the tensors it was captured with; load new data into them in place
    (copy_) before a replay.
Gradients of parameters that the optimizer does not own (the frozen wav2vec2 weights, as in the
reference) keep accumulating in their .grad buffers across replays, exactly as in eager steps.

Segmented capture (segmented=True, the data-parallel step): a collective cannot live inside a graph,
so every host collective the step issues through functional.collective() — the SyncBN statistics
all-reduces of the Conformer's conv modules (forward and backward) and the gradient-bucket all-reduces
as buckets complete — ends the graph captured so far and starts the next. The segments share one
memory pool (replayed in capture order, as the pool requires); a replay runs segment 0, the first
collective, segment 1, ... so a bucket's RCCL all-reduce (async) runs beside the rest of the
backward.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .. import _lib
from .. import functional as Fn


# One capture stream per (device, priority) for the whole process: every stream takes one of the few
# hardware queues a process gets (GPU_MAX_HW_QUEUES, 4 by default), so captures (one per batch shape,
# one per model) share it instead of each opening another.
_CAPTURE_STREAMS: dict = {}

# The step counter the library's dropout kernels currently read (b2p_set_seed_epoch keeps a raw device
# pointer): held here so the tensor outlives every StepGraph that shares it. Without this reference a
# Trainer collected without release() left the library pointing at freed memory, and the next eager
# kernels read whatever tensor the allocator put there (two dropout launches with one seed drew
# different masks).
_INSTALLED_EPOCH = [None]


def _install_epoch(t) -> None:
    _lib.check(_lib.load().b2p_set_seed_epoch(None if t is None else ctypes.c_void_p(t.data_ptr())),
               "b2p_set_seed_epoch")
    _INSTALLED_EPOCH[0] = t


def live_graph_nodes(module_prefix: str = "wav2vec2forbrain_amd") -> int:
    """Number of live autograd nodes of custom Functions defined under module_prefix (the backward
    contexts of this package's fused ops). A node outlives its step when the caller still holds a
    graph output (a loss or logits with grad_fn) or retained the graph; capturing a step then
    segfaulted inside hipStreamEndCapture (round 3, test_trainer_replay_matches_eager)."""
    import gc
    gc.collect()
    n = 0
    for o in gc.get_objects():
        if isinstance(o, torch.autograd.function.BackwardCFunction):
            cls = getattr(o, "_forward_cls", None)
            if cls is not None and cls.__module__.startswith(module_prefix):
                n += 1
    return n


def _capture_stream(dev, prio: bool):
    key = (str(dev), prio)
    s = _CAPTURE_STREAMS.get(key)
    if s is None:
        s = _CAPTURE_STREAMS[key] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1]
                                                      if prio else 0)
    return s


class _SegmentedCapture:
    """Graphs captured back to back on one stream and one memory pool, split at host collectives."""

    def __init__(self, stream):
        self.stream = stream
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: list = []
        self.calls: list = []
        self.cur = None

    def begin(self) -> None:
        g = torch.cuda.CUDAGraph()
        # relaxed: a split inside the backward begins the next segment on autograd's worker thread
        # and the main thread ends it (the other modes tie a capture to the thread that began it)
        with torch.cuda.stream(self.stream):
            g.capture_begin(pool=self.pool, capture_error_mode="relaxed")
        self.cur = g

    def end(self) -> None:
        if self.cur is None:   # an error between a split's end() and its begin(): nothing is capturing
            return
        with torch.cuda.stream(self.stream):
            self.cur.capture_end()
        self.graphs.append(self.cur)
        self.cur = None

    def split(self, fn) -> None:
        self.end()
        self.calls.append(fn)
        self.begin()

    def replay(self) -> None:
        n = len(self.graphs)
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.calls):
                Fn._Segments.remaining = n - 1 - i
                try:
                    self.calls[i]()
                finally:
                    Fn._Segments.remaining = 0

    def reset(self) -> None:
        for g in self.graphs:
            g.reset()
        self.graphs, self.calls = [], []


class StepGraph:
    def __init__(self, step_fn, optimizer=None, warmup: int = 2, warm_replays: int = 2, epoch=None,
                 segmented: bool = False):
        """step_fn() runs one step on the current stream and returns the loss tensor (no host
        syncs inside: model.sync_metrics must be False). Pass the optimizer when step_fn includes
        its update (captured); without it the update runs eagerly after each replay (the data-
        parallel step: replay, gradient all-reduce, update). epoch: a shared int64 device step
        counter (several graphs of one training run, e.g. one per batch shape, draw from one
        dropout-seed sequence); a new one by default."""
        self.step_fn = step_fn
        self.opt = optimizer
        self.warmup = warmup
        self.warm_replays = warm_replays
        self.graph = None
        self.loss = None
        self.epoch = epoch
        self.segmented = segmented
        self.pin = None        # the reserved column-sum counter ranges (b2p_colsum_pin_end id)

    def capture(self) -> None:
        live = live_graph_nodes()
        if live:
            raise RuntimeError(
                f"StepGraph.capture: {live} autograd nodes of an earlier step are still alive (an output "
                "with grad_fn is held, or a graph was retained); detach or drop them before capturing")
        dev = torch.device("cuda", torch.cuda.current_device())
        lib = _lib.load()
        if self.epoch is None:
            self.epoch = torch.zeros(1, dtype=torch.int64, device=dev)
        _install_epoch(self.epoch)
        if self.opt is not None:
            self.opt.make_capturable(dev)
        Fn.set_gemm_timing(False)
        # the capture stream at normal priority (B2P_GRAPH_PRIORITY=1: the highest). A high-priority
        # capture stream measured the same for the first graph of a process, but every graph captured
        # after it replayed far slower (Conformer-large step 154 ms instead of 88 ms: the base run's
        # graph before it in bench.py, or any earlier capture; tools/nested_probe.py, graph_probe.py)
        prio = int(os.environ.get("B2P_GRAPH_PRIORITY", "0"))
        s = _capture_stream(dev, bool(prio))
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):         # allocator / side-stream warm-up on the capture stream
                self._one()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # the host side of the captured step runs once now without updating anything: keep the
        # optimizer's host step counters as they were (after_replay advances them per replay)
        steps = ({p: st["step"].clone() for p, st in self.opt.state.items() if "step" in st}
                 if self.opt is not None else {})
        # the column-sum arrival counters this capture's launches take stay reserved while it lives
        _lib.check(lib.b2p_colsum_pin_begin(), "b2p_colsum_pin_begin")
        try:
            self._capture_graph(s)
        except BaseException:
            lib.b2p_colsum_unpin(lib.b2p_colsum_pin_end())
            raise
        self.pin = lib.b2p_colsum_pin_end()
        torch.cuda.synchronize()
        for p, t in steps.items():
            self.opt.state[p]["step"] = t
        for _ in range(self.warm_replays):   # first launches of a new graph pay its upload
            self.replay()
        torch.cuda.synchronize()

    def _capture_graph(self, s) -> None:
        if self.segmented:
            g = _SegmentedCapture(s)
            Fn._Segments.active = g
            g.begin()
            try:
                with torch.cuda.stream(s):
                    self.loss = self._one()
            except BaseException:
                Fn._Segments.active = None
                try:
                    g.end()
                finally:
                    g.reset()
                raise
            Fn._Segments.active = None
            g.end()
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self.loss = self._one()
        self.graph = g

    def _one(self):
        _lib.check(_lib.load().b2p_seed_epoch_step(ctypes.c_void_p(self.epoch.data_ptr()),
                                                   ctypes.c_void_p(_lib.stream_ptr())), "b2p_seed_epoch_step")
        return self.step_fn()

    def replay(self) -> torch.Tensor:
        """One training step; returns the (static) loss tensor — clone it to keep the value."""
        if self.opt is not None:
            self.opt.prepare_replay()
        self.graph.replay()     # a CUDAGraph, or a _SegmentedCapture (segments and the collectives between)
        if self.opt is not None:
            self.opt.after_replay()
        return self.loss

    @property
    def segments(self) -> int:
        """Graphs one replay runs (1 unless segmented)."""
        if self.graph is None:
            return 0
        return len(self.graph.graphs) if self.segmented else 1

    def release(self) -> None:
        """Back to eager semantics (the seed counter is no longer mixed in); the executable graph and
        its resources are destroyed now rather than whenever the Python object is collected."""
        _install_epoch(None)
        if self.graph is not None:
            torch.cuda.synchronize()
            self.graph.reset()
        if self.pin is not None:
            _lib.load().b2p_colsum_unpin(self.pin)
            self.pin = None
        self.graph = None
        self.loss = None
