"""HipAdam: torch.optim.Adam-compatible optimizer whose update runs in the multi-tensor HIP kernel
(b2p_adam_multi). Same hyper-parameters, param-group semantics, state names (step, exp_avg,
exp_avg_sq) and numerics as torch.optim.Adam (amsgrad=False, maximize=False) — the optimizer the
reference builds in src/experiments/experiment.py:25-28 / b2t_gru_w2v_experiment.py:138-145,
so LR schedulers (StepLR, LambdaLR warmup) and state_dict round-trips work unchanged."""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from . import functional as Fn


class HipAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, **kw):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by the reference")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.capturable = False
        self._dev = []       # per param group: (lr float32[1], step float64[1], hyper float32[3]) on device

    def make_capturable(self, device) -> None:
        """Switch to the graph-replayable update (b2p_adam_multi_dev: lr and the step counter live on
        the device, the bias corrections are formed there). Call before capturing a step; then call
        prepare_replay() before and after_replay() after every replay."""
        self._dev = []
        for group in self.param_groups:
            steps = [float(self.state[p]["step"]) for p in group["params"] if len(self.state[p])]
            t = steps[0] if steps else 0.0
            self._dev.append((torch.full((1,), float(group["lr"]), device=device, dtype=torch.float32),
                              torch.full((1,), t, device=device, dtype=torch.float64),
                              torch.zeros(3, device=device, dtype=torch.float32)))
        self.capturable = True

    def prepare_replay(self) -> None:
        """Stream-ordered refresh of each group's device lr (LR schedulers change it on the host)."""
        for group, (lr, _, _) in zip(self.param_groups, self._dev):
            lr.fill_(float(group["lr"]))

    def after_replay(self) -> None:
        """Host-side step counters (state_dict) advance with every replayed update, and cached bf16
        copies of the updated parameters are invalidated."""
        for group in self.param_groups:
            ps = []
            for p in group["params"]:
                st = self.state[p]
                if len(st):
                    st["step"] += 1
                    ps.append(p)
            Fn.bump_param_epoch(ps)

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
                arr = (ctypes.c_int64 * len(recs))(*recs)
                if self.capturable:
                    if len(buckets) != 1:
                        raise RuntimeError("HipAdam(capturable): a param group's tensors must share one step count")
                    lr_d, step_d, hyp_d = self._dev[self.param_groups.index(group)]
                    _lib.check(lib.b2p_adam_recs(arr, len(ps), 0.0, float(b1), float(b2), float(group["eps"]),
                                                 float(group["weight_decay"]), 1.0, 1.0, lr_d.data_ptr(),
                                                 step_d.data_ptr(), hyp_d.data_ptr(), stream), "b2p_adam_recs")
                else:
                    bc1 = 1.0 - b1 ** step
                    bc2s = math.sqrt(1.0 - b2 ** step)
                    _lib.check(lib.b2p_adam_recs(arr, len(ps), float(group["lr"]), float(b1), float(b2),
                                                 float(group["eps"]), float(group["weight_decay"]), float(bc1),
                                                 float(bc2s), None, None, None, stream), "b2p_adam_recs")
                Fn.bump_param_epoch(ps)   # in-place writes invisible to torch: drop bf16 weight copies
        return loss
