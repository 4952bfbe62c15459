"""Data-parallel gradient exchange for the b2p2t training step: one process per GPU,
torch.distributed over RCCL (backend "nccl" on ROCm) / gloo on CPU.

GradBucketReducer packs the trainable gradients into fixed buckets in reverse registration order
(lm_head -> encoder layers -> fc -> GRU -> front end, i.e. the order backward produces them) and
issues an async all-reduce per bucket from the post-accumulate-grad hook as soon as the bucket is
complete, so the exchange overlaps the rest of the backward. Buckets are static: a parameter that
got no gradient on this rank (LayerDrop-skipped layer) contributes zeros, never a "find unused
parameters" pass. Parameters that the path never uses (reference inpLayer*, hidden_start unless
learnable, conformer pos_conv_embed) are excluded by the caller.

Bucket size: the xGMI fabric of an MI355X node is point-to-point (7 links x ~153 GB/s per GPU);
RCCL spreads one large all-reduce over all links with multiple channels, so fewer, larger buckets
(default 64 MB) amortise the per-collective latency while still leaving >= 2 buckets to overlap
for the 64 MB frozen-w2v gradient set.
"""
from __future__ import annotations

from typing import Iterable

import torch
import torch.distributed as dist


class GradBucketReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 64.0, process_group=None,
                 average: bool = True, overlap: bool = True):
        self.params = [p for p in params if p.requires_grad]
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.average = average
        # overlap=False: no collective from the backward hooks, finish() exchanges every bucket (the
        # graph-replayed step: backward is captured, the RCCL exchange runs after each replay)
        self.overlap = overlap
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
        self.offsets = {}
        self.flat = []
        for bi, b in enumerate(self.buckets):
            off = 0
            for p in b:
                self.bucket_of[p] = bi
                self.offsets[p] = off
                off += p.numel()
            dev = b[0].device
            self.flat.append(torch.empty(off, device=dev, dtype=torch.float32))
        self._handles = []
        self._reset()
        if self.world > 1:
            for p in self.params:
                p.register_post_accumulate_grad_hook(self._hook)

    def _reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = [None] * len(self.buckets)

    def _launch(self, bi: int):
        flat = self.flat[bi]
        for p in self.buckets[bi]:
            o = self.offsets[p]
            seg = flat[o:o + p.numel()]
            if p.grad is None:
                seg.zero_()
            else:
                seg.copy_(p.grad.reshape(-1))
        self.works[bi] = dist.all_reduce(flat, group=self.pg, async_op=True)
        self.launched[bi] = True

    def _hook(self, p):
        if not self.overlap:
            return
        bi = self.bucket_of.get(p)
        if bi is None or self.launched[bi]:
            return
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            self._launch(bi)

    def finish(self):
        """Call after loss.backward(): launches incomplete buckets, waits, writes averaged grads."""
        if self.world <= 1:
            return
        for bi in range(len(self.buckets)):
            if not self.launched[bi]:
                self._launch(bi)
        for bi, w in enumerate(self.works):
            w.wait()
            flat = self.flat[bi]
            if self.average:
                flat.div_(self.world)
            for p in self.buckets[bi]:
                o = self.offsets[p]
                g = flat[o:o + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
        self._reset()


def unused_param_names(model: torch.nn.Module) -> set[str]:
    """Parameters the training path never touches (reference quirks)."""
    out = set()
    for n, _ in model.named_parameters():
        if ".inpLayer" in n or n.startswith("inpLayer"):
            out.add(n)
        if n.endswith("hidden_start"):
            enc = model
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
