"""HipAdam: torch.optim.Adam-compatible optimizer whose update runs in the multi-tensor HIP kernel
(b2p_adam_multi). Same hyper-parameters, param-group semantics, state names (step, exp_avg,
exp_avg_sq) and numerics as torch.optim.Adam (amsgrad=False, maximize=False) — the optimizer the
reference builds in src/experiments/experiment.py:25-28 / b2t_gru_w2v_experiment.py:138-145,
so LR schedulers (StepLR, LambdaLR warmup) and state_dict round-trips work unchanged."""
from __future__ import annotations

import math

import torch

from . import _lib
from . import functional as Fn


class HipAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, **kw):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by the reference")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = {}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        Fn.join_wgrad()    # deferred frozen-parameter gradient work is ordered before the update
        lib = _lib.load()
        stream = _lib.stream_ptr()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            # bucket by step count (identical for all params of a group in practice)
            buckets: dict[int, list] = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("HipAdam does not support sparse gradients")
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()
                        and p.grad.dtype == torch.float32):
                    raise RuntimeError("HipAdam expects contiguous fp32 device parameters and gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                buckets.setdefault(int(st["step"].item()), []).append(p)
            for step, ps in buckets.items():
                recs = []
                maxn = 0
                for p in ps:
                    st = self.state[p]
                    recs += [p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             p.numel()]
                    maxn = max(maxn, p.numel())
                key = tuple(recs)
                table = self._tables.get(key)
                if table is None:
                    table = torch.tensor(recs, dtype=torch.int64).to(ps[0].device, non_blocking=False)
                    if len(self._tables) > 64:
                        self._tables.clear()
                    self._tables[key] = table
                bc1 = 1.0 - b1 ** step
                bc2s = math.sqrt(1.0 - b2 ** step)
                _lib.check(lib.b2p_adam_multi(table.data_ptr(), len(ps), maxn, float(group["lr"]), float(b1),
                                              float(b2), float(group["eps"]), float(group["weight_decay"]),
                                              float(bc1), float(bc2s), stream), "b2p_adam_multi")
                Fn.bump_param_epoch(ps)   # in-place writes invisible to torch: drop bf16 weight copies
        return loss
