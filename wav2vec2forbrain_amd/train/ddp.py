"""Data-parallel gradient exchange for the b2p2t training step: one process per GPU,
torch.distributed over RCCL (backend "nccl" on ROCm) / gloo on CPU.

GradBucketReducer packs the trainable gradients into fixed buckets in reverse registration order
(lm_head -> encoder layers -> fc -> GRU -> front end, i.e. the order backward produces them). The
gradients live IN the buckets: zero_grad() binds every p.grad to its slice of a flat bucket buffer,
so autograd accumulates straight into the buffer that is all-reduced (no copy in, no copy out).
Buckets are launched strictly in index order on every rank (bucket i only after buckets < i), as
from the post-accumulate-grad hook as soon as they are complete, so the exchange overlaps the rest
of the backward and the collectives match across ranks even when a rank's backward skips a
parameter (LayerDrop): such a parameter contributes the zeros of its bucket slice. Parameters the
path never uses (reference inpLayer*, hidden_start unless learnable, conformer pos_conv_embed) are
excluded by the caller.

Bucket size: the xGMI fabric of an MI355X node is point-to-point (7 links x ~153 GB/s per GPU);
RCCL spreads one large all-reduce over all links with multiple channels, so fewer, larger buckets
(default 64 MB) amortise the per-collective latency while still leaving several buckets to overlap
for the full-fine-tune gradient sets (424 MB base, 2.47 GB Conformer-large).

Graph-replayed steps over RCCL (the default for NCCL process groups, collectives_in_graph): the whole
step is one graph. The backward hooks launch each bucket's all-reduce while the capture runs, so every
replay issues it on RCCL's stream as soon as the bucket's last gradient is accumulated, beside the rest
of the backward; the tail (remaining buckets, the used-flag MAX, the waits, the clip) and the Adam update
are captured too, so a replay is one host call for the whole data-parallel step. gloo (host collectives):
a bucket's launch goes through functional.collective(), so inside a segmented capture
(train/step_graph.py) it splits the captured step there and each replay issues the bucket's all-reduce
between the segments (full fine-tuning, config 5); with frozen-weight gradients on the side streams
(configs 1-4) the buckets are exchanged after the replay, since a split would join those streams mid-GRU.
"""
from __future__ import annotations

from typing import Iterable

import os
from collections import deque

import torch
import torch.distributed as dist

from .. import functional as Fn


def dp_active(process_group=None) -> bool:
    """The data-parallel machinery is on: torch.distributed initialised with more than one rank, or with
    one rank under B2P_DP_FORCE=1 (tests: the RCCL path of every collective on a one-GPU box)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(process_group) > 1 or os.environ.get("B2P_DP_FORCE") == "1"


def collectives_in_graph(process_group=None) -> bool:
    """Captured data-parallel steps keep their collectives INSIDE the graph (RCCL all-reduces captured
    as graph nodes: one graph per step instead of one segment per collective). RCCL only (gloo
    collectives are host code); B2P_GRAPH_COLLECTIVES=0 keeps the segmented capture for RCCL too."""
    return (dp_active(process_group) and dist.get_backend(process_group) == "nccl"
            and os.environ.get("B2P_GRAPH_COLLECTIVES", "1") != "0")


class GradBucketReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 64.0, process_group=None,
                 average: bool = True, overlap: bool = True, grad_views: bool = True, track_used: bool = True):
        self.params = [p for p in params if p.requires_grad]
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.active = dp_active(process_group)
        self.average = average
        # RCCL averages inside the collective; gloo has no AVG: sum, then one scale
        self.avg_op = (average and dist.is_initialized()
                       and dist.get_backend(process_group) == "nccl")
        # overlap=False: no collective from the backward hooks, finish() exchanges every bucket (the
        # graph-replayed step: backward is captured, the RCCL exchange runs after each replay)
        self.overlap = overlap
        self.grad_views = grad_views
        cap = int(bucket_mb * 1024 * 1024 / 4)
        self.buckets: list[list[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel()
            if size >= cap:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {}
        self.views = {}
        self.flat = []
        for bi, b in enumerate(self.buckets):
            n = sum(p.numel() for p in b)
            flat = torch.zeros(n, device=b[0].device, dtype=torch.float32)
            off = 0
            for p in b:
                self.bucket_of[p] = bi
                self.views[p] = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            self.flat.append(flat)
        # diagnostics (bounded: a long run issues ~40 bucket launches per step)
        self.launch_log: deque = deque(maxlen=4096)    # bucket indices in the order their collectives were issued
        # per launch: the captured segments a replay still ran after it (> 0: overlapped the backward)
        self.launch_tail: deque = deque(maxlen=4096)
        self.launch_pending: deque = deque(maxlen=4096)
        # "used by some rank this step" per parameter (int32, MAX-reduced in finish()): the gates
        # HipAdam's device form reads (opt.gates = reducer.gates), so a parameter no rank used —
        # every rank's LayerDrop dropped its layer — is left untouched, as torch.optim.Adam leaves a
        # grad=None parameter of the reference's single process
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.used = torch.ones(max(len(self.params), 1), dtype=torch.int32, device=dev)
        self.gates = {id(p): self.used[k] for k, p in enumerate(self.params)}
        # track_used=False (frozen parameters: nobody reads their gates, their gradients come from the
        # deferred GEMMs, not from autograd hooks): no flag exchange at all
        self.track_used = track_used
        # eager steps: the local flags go up through a persistent pinned buffer (stream-ordered copy; the
        # event guards the buffer against being refilled before the previous step's copy has run)
        self._loc_host = (torch.ones(max(len(self.params), 1), dtype=torch.int32).pin_memory()
                          if dev.type == "cuda" else None)
        self._loc_event = None
        self._idx_host = (torch.zeros(max(len(self.params), 1), dtype=torch.int64).pin_memory()
                          if dev.type == "cuda" else None)
        self._pos = {id(p): k for k, p in enumerate(self.params)}
        self._layer_gates = None   # graph-replayed steps: the device LayerDrop flags (make_layer_gates)
        self._seen: set = set()
        self._reset()
        self._hooks = []
        if self.active:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._hook))
        if grad_views:
            self.zero_grad()

    def close(self) -> None:
        """Detaches this reducer from its parameters (backward hooks removed, gradients unbound from the
        bucket views), so another reducer can take them over (the Trainer rebuilds its reducers when
        the optimizer gains a param group)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.grad_views:
            for p in self.params:
                if p.grad is not None and p.grad.data_ptr() == self.views[p].data_ptr():
                    p.grad = None
        self.active = False

    def make_layer_gates(self, param_flags: dict):
        """Graph-replayed steps (backward captured: no hook fires on a replay): the local "used" flag
        of each parameter is its layer's device LayerDrop flag of the captured step
        ({id(p): int32 flag}, functional.layerdrop_param_gates()); other parameters are always used.
        Returns the state to pass to use_layer_gates() before each replay's finish()."""
        flags, src = [], []
        for p in self.params:
            f = param_flags.get(id(p))
            if f is None:
                src.append(-1)
            else:
                for j, g in enumerate(flags):
                    if g is f:
                        src.append(j)
                        break
                else:
                    flags.append(f)
                    src.append(len(flags) - 1)
        # no LayerDrop flag at all (deterministic mode / no dropped layers): every parameter is
        # used — a replay fires no backward hook, so the hook-based flags would all read "unused"
        one = torch.ones(1, dtype=torch.int32, device=self.used.device)
        vals = [len(flags) if s < 0 else s for s in src]
        if self._idx_host is not None:
            # a stream-ordered copy from the pinned buffer allocated with the reducer: the RCCL step calls
            # this inside its capture, where no host memory can be pinned (every capture writes the same
            # mapping: a parameter's layer does not change)
            self._idx_host[:len(vals)] = torch.tensor(vals, dtype=torch.int64)
            idx = self._idx_host[:len(vals)].to(self.used.device, non_blocking=True)
        else:
            idx = torch.tensor(vals, dtype=torch.int64, device=self.used.device)
        return (flags + [one], idx)

    def use_layer_gates(self, state) -> None:
        """None: the local used flags come from the backward hooks (eager steps)."""
        self._layer_gates = state

    def _reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.next_launch = 0
        self.works = [None] * len(self.buckets)
        self._seen = set()

    def _exchange_used(self):
        """Local used flags -> MAX over ranks into self.used (the optimizer's gates)."""
        if not self.params:
            return
        if not self.track_used:
            return
        if self._layer_gates is not None:
            flags, idx = self._layer_gates
            torch.index_select(torch.cat([f.reshape(1) for f in flags]), 0, idx, out=self.used)
        elif self._loc_host is not None:
            if self._loc_event is not None:
                self._loc_event.synchronize()
            loc = self._loc_host.numpy()
            loc[:] = 0
            loc[[self._pos[i] for i in self._seen if i in self._pos]] = 1
            self.used.copy_(self._loc_host, non_blocking=True)
            self._loc_event = torch.cuda.Event()
            self._loc_event.record()
        else:
            loc = torch.tensor([1 if id(p) in self._seen else 0 for p in self.params], dtype=torch.int32)
            self.used.copy_(loc)
        if self.active:
            dist.all_reduce(self.used, op=dist.ReduceOp.MAX, group=self.pg)

    def zero_grad(self) -> None:
        """Zeroes the buckets and binds every p.grad to its bucket slice (use instead of the
        optimizer's zero_grad for these parameters: set_to_none would unbind the views)."""
        for f in self.flat:
            f.zero_()
        if self.grad_views:
            for p in self.params:
                if p.grad is None or p.grad.data_ptr() != self.views[p].data_ptr():
                    p.grad = self.views[p]

    def _launch(self, bi: int):
        for p in self.buckets[bi]:
            v = self.views[p]
            if p.grad is None:
                v.zero_()
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
        op = dist.ReduceOp.AVG if self.avg_op else dist.ReduceOp.SUM
        self.works[bi] = dist.all_reduce(self.flat[bi], op=op, group=self.pg, async_op=True)
        self.launch_log.append(bi)
        self.launch_tail.append(Fn.segments_remaining())
        # parameters whose gradient was still to come when this bucket went out (> 0: issued mid-backward)
        self.launch_pending.append(len(self.params) - len(self._seen))

    def _launch_all(self, bis):
        for bi in bis:
            self._launch(bi)
        self.next_launch = max(self.next_launch, bis[-1] + 1)

    def _launch_ready(self):
        ready = []
        while self.next_launch < len(self.buckets) and self.pending[self.next_launch] == 0:
            ready.append(self.next_launch)
            self.next_launch += 1
        if ready:
            # eager: now; segmented capture: between the segments of every replay
            Fn.collective(lambda: self._launch_all(ready))

    def _hook(self, p):
        self._seen.add(id(p))
        if not self.overlap:
            return
        bi = self.bucket_of.get(p)
        if bi is None or bi < self.next_launch:
            return
        self.pending[bi] -= 1
        self._launch_ready()

    def finish(self):
        """Call after loss.backward(): launches the remaining buckets (in order), waits, and leaves
        the averaged gradient in every p.grad (its bucket slice)."""
        if not self.active:
            return
        while self.next_launch < len(self.buckets):
            self._launch(self.next_launch)
            self.next_launch += 1
        self._exchange_used()
        for bi, w in enumerate(self.works):
            w.wait()
            if self.average and not self.avg_op:
                self.flat[bi].div_(self.world)
            for p in self.buckets[bi]:
                if p.grad is None or p.grad.data_ptr() != self.views[p].data_ptr():
                    p.grad = self.views[p]
        self._reset()


def unused_param_names(model: torch.nn.Module) -> set[str]:
    """Parameters the training path never touches (reference quirks)."""
    out = set()
    for n, _ in model.named_parameters():
        if ".inpLayer" in n or n.startswith("inpLayer"):
            out.add(n)
        if n.endswith("hidden_start"):
            learn = False
            try:
                learn = model.brain_encoder.neural_decoder.encoder.config.encoder_learnable_inital_state
            except AttributeError:
                pass
            if not learn:
                out.add(n)
        if "wav2vec2_conformer.encoder.pos_conv_embed" in n:
            out.add(n)
    return out


def allreduce_mean_scalar(x: torch.Tensor, process_group=None) -> torch.Tensor:
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return x
    y = x.detach().clone()
    dist.all_reduce(y, group=process_group)
    return y / dist.get_world_size(process_group)
