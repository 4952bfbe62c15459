"""HipAdam: torch.optim.Adam-compatible optimizer whose update runs in the multi-tensor HIP kernels
(csrc/adam.hip). Same hyper-parameters, param-group semantics, state names (step, exp_avg,
exp_avg_sq) and numerics as torch.optim.Adam (amsgrad=False, maximize=False) — the optimizer the
reference builds in src/experiments/experiment.py:25-28 / b2t_gru_w2v_experiment.py:138-145,
so LR schedulers (StepLR, LambdaLR warmup) and state_dict round-trips work unchanged.

Two forms:
  * host form (default): lr and the bias corrections are formed on the host per step, like
    torch.optim.Adam; a parameter whose .grad is None is skipped.
  * device form (make_capturable: captured / graph-replayed and data-parallel steps): every
    parameter owns a device step counter, lr lives on the device, and each tensor may carry a device
    gate (int32, 0 = leave the parameter untouched this step). torch.optim.Adam skips a parameter
    whose .grad is None — no moment update, no weight decay, no step increment. Under LayerDrop the
    reference never runs a dropped layer, so its parameters are such None-grad parameters; a captured
    step runs every layer and hands the layer's gate (functional.layerdrop_param_gates) to the
    update instead, and a data-parallel step hands the gate "some rank used it"
    (train.ddp.GradBucketReducer.gates), so both leave exactly the reference's parameters alone.
"""
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
        # device form, per param group: lr float32[1], per-parameter step counters float64[n],
        # hyper scratch float32[4n], {id(p): index}
        self._dev = []
        # optional {id(p): int32 device tensor}: the caller's per-parameter gates (data-parallel
        # steps: 0 = no rank used the parameter this step); device form only
        self.gates = None

    # ------------------------------------------------------------------ device form
    def make_capturable(self, device) -> None:
        """Switch to the device form (graph-replayable update with per-parameter device step counters
        and gates). Call before capturing a step; then call prepare_replay() before and
        after_replay() after every replay. State is created here for every trainable parameter (zero
        moments, step 0: what torch.optim.Adam creates at a parameter's first gradient), so nothing
        is allocated inside a captured step. Idempotent: captured steps hold pointers to the device
        counters, so a second call (another capture) keeps them."""
        if self.capturable:
            return
        self._dev = []
        for group in self.param_groups:
            ps = group["params"]
            for p in ps:
                st = self.state[p]
                if len(st) == 0 and p.requires_grad:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            steps = [float(self.state[p]["step"]) if len(self.state[p]) else 0.0 for p in ps]
            self._dev.append(dict(
                lr=torch.full((1,), float(group["lr"]), device=device, dtype=torch.float32),
                steps=torch.tensor(steps, device=device, dtype=torch.float64),
                hyper=torch.zeros(4 * max(len(ps), 1), device=device, dtype=torch.float32),
                index={id(p): i for i, p in enumerate(ps)}))
        self.capturable = True

    def sync_steps(self) -> None:
        """Copies the device step counters into the host state (state_dict, inspection)."""
        if not self.capturable:
            return
        for group, d in zip(self.param_groups, self._dev):
            host = d["steps"].cpu().tolist()
            for p in group["params"]:
                st = self.state[p]
                if len(st):
                    st["step"] = torch.tensor(float(host[d["index"][id(p)]]))

    def state_dict(self):
        self.sync_steps()
        sd = super().state_dict()
        if self.capturable:
            # the device form creates state for every trainable parameter up front; torch.optim.Adam
            # has none for a parameter that never received a gradient (unused inpLayer* etc.)
            sd["state"] = {k: v for k, v in sd["state"].items() if float(v["step"]) > 0}
        return sd

    def load_state_dict(self, state_dict) -> None:
        """Device form: captured steps hold raw pointers to the moment tensors and step counters, so the
        loaded values are copied INTO the existing tensors (the pointers stay valid and graphs captured
        before the load replay from the loaded state). A trainable parameter absent from the loaded
        state (torch.optim.Adam keeps none for a parameter that never had a gradient, and state_dict()
        drops step-0 entries) gets zero moments and step 0 again, as make_capturable() creates them."""
        if not self.capturable:
            super().load_state_dict(state_dict)
            return
        keep = {p: (st.get("exp_avg"), st.get("exp_avg_sq")) for p, st in self.state.items() if len(st)}
        super().load_state_dict(state_dict)
        for group, d in zip(self.param_groups, self._dev):
            for p in group["params"]:
                old = keep.get(p)
                st = self.state[p]
                if old is None or old[0] is None:
                    if p.requires_grad and len(st) == 0:
                        raise RuntimeError("HipAdam (device form): a trainable parameter without device state")
                    continue
                ea, eas = old
                if len(st):
                    ea.copy_(st["exp_avg"])
                    eas.copy_(st["exp_avg_sq"])
                else:
                    ea.zero_()
                    eas.zero_()
                    st["step"] = torch.tensor(0.0)
                st["exp_avg"], st["exp_avg_sq"] = ea, eas
            steps = [float(self.state[p]["step"]) if len(self.state[p]) else 0.0 for p in group["params"]]
            d["steps"].copy_(torch.tensor(steps, dtype=torch.float64))

    def add_param_group(self, param_group) -> None:
        """torch.optim.Optimizer.add_param_group; in the device form the new group gets its device lr,
        step counters and state right away. A step captured BEFORE this call holds update records for
        the old groups only: `generation` advances, and the Trainer re-captures its cached steps when it
        sees a new generation (train_loop.Trainer.train_step)."""
        super().add_param_group(param_group)
        self.generation = getattr(self, "generation", 0) + 1
        if getattr(self, "capturable", False):
            self.capturable = False
            dev, self._dev = self._dev, []
            device = dev[0]["lr"].device if dev else self.param_groups[0]["params"][0].device
            self.make_capturable(device)
            # the existing groups keep their device tensors (captured steps point at them)
            self._dev[:len(dev)] = dev

    def prepare_replay(self) -> None:
        """Stream-ordered refresh of each group's device lr (LR schedulers change it on the host)."""
        for group, d in zip(self.param_groups, self._dev):
            d["lr"].fill_(float(group["lr"]))

    def after_replay(self) -> None:
        """Cached 16-bit copies of the updated parameters are invalidated (the device step counters
        advanced inside the replay; sync_steps() brings them to the host state)."""
        for group in self.param_groups:
            Fn.bump_param_epoch([p for p in group["params"] if len(self.state[p])])

    def _gate_of(self, p, ld_gates):
        if self.gates is not None and id(p) in self.gates:
            return self.gates[id(p)].data_ptr()
        f = ld_gates.get(id(p))
        return f.data_ptr() if f is not None else 0

    def _step_device(self, lib, stream):
        if len(self._dev) != len(self.param_groups):
            raise RuntimeError("HipAdam (device form): param groups without device state")
        capturing = Fn.capturing()
        ld_gates = Fn.layerdrop_param_gates() if capturing else {}
        for group, d in zip(self.param_groups, self._dev):
            b1, b2 = group["betas"]
            if not capturing:   # inside a capture prepare_replay() refreshes lr before every replay
                d["lr"].fill_(float(group["lr"]))
            recs, ps = [], []
            base = d["steps"].data_ptr()
            for p in group["params"]:
                if p.grad is None:
                    continue
                self._check(p)
                st = self.state[p]
                if len(st) == 0:
                    raise RuntimeError("HipAdam (device form): a parameter without optimizer state got a "
                                       "gradient; call make_capturable() after adding parameters")
                recs += [p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                         p.numel(), base + 8 * d["index"][id(p)], self._gate_of(p, ld_gates)]
                ps.append(p)
            if not ps:
                continue
            arr = (ctypes.c_int64 * len(recs))(*recs)
            _lib.check(lib.b2p_adam_gated_recs(arr, len(ps), d["lr"].data_ptr(), float(b1), float(b2),
                                               float(group["eps"]), float(group["weight_decay"]),
                                               d["hyper"].data_ptr(), stream), "b2p_adam_gated_recs")
            Fn.bump_param_epoch(ps)

    @staticmethod
    def _check(p):
        if p.grad.is_sparse:
            raise RuntimeError("HipAdam does not support sparse gradients")
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()
                and p.grad.dtype == torch.float32):
            raise RuntimeError("HipAdam expects contiguous fp32 device parameters and gradients")

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        Fn.join_wgrad()    # deferred frozen-parameter gradient work is ordered before the update
        lib = _lib.load()
        stream = _lib.stream_ptr()
        if self.capturable:
            self._step_device(lib, stream)
            return loss
        for group in self.param_groups:
            b1, b2 = group["betas"]
            # bucket by step count (identical for all params of a group in practice)
            buckets: dict[int, list] = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                self._check(p)
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                buckets.setdefault(int(st["step"].item()), []).append(p)
            for step, ps in buckets.items():
                recs = []
                for p in ps:
                    st = self.state[p]
                    recs += [p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                             p.numel()]
                arr = (ctypes.c_int64 * len(recs))(*recs)
                bc1 = 1.0 - b1 ** step
                bc2s = math.sqrt(1.0 - b2 ** step)
                _lib.check(lib.b2p_adam_recs(arr, len(ps), float(group["lr"]), float(b1), float(b2),
                                             float(group["eps"]), float(group["weight_decay"]), float(bc1),
                                             float(bc2s), None, None, None, stream), "b2p_adam_recs")
                Fn.bump_param_epoch(ps)   # in-place writes invisible to torch: drop bf16 weight copies
        return loss
