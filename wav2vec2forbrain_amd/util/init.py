"""Deterministic, order-independent parameter initialisation shared by tests, golden-fixture
generation and bench.py (random-init weights of the reference architecture; the pretrained hub
checkpoints are unreachable offline). Each tensor is drawn from a CPU torch.Generator seeded with
(seed, crc32(name)), so the same name/shape gives the same values on every machine with this
torch build, independent of module construction order."""
from __future__ import annotations

import zlib

import torch


def _value(name: str, shape, seed: int) -> torch.Tensor:
    g = torch.Generator()
    g.manual_seed((seed * 1000003 + zlib.crc32(name.encode())) & 0x7FFFFFFFFFFFFFFF)
    r = torch.randn(*shape, generator=g, dtype=torch.float32)
    if name.endswith("day_weights"):
        return torch.eye(shape[-1]).expand(*shape).clone() + 0.05 * r
    if name.endswith("day_bias"):
        return 0.1 * r
    if "layer_norm.weight" in name or name.endswith("norm.weight"):
        return 1.0 + 0.1 * r
    if name.endswith("parametrizations.weight.original0"):
        return 1.0 + 0.1 * r
    if name.endswith("parametrizations.weight.original1") or name.endswith("hidden_start"):
        return r
    if name.endswith("bias") or len(shape) < 2:
        return 0.05 * r
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    return r / fan_in ** 0.5


def deterministic_state(named_shapes, seed: int = 42) -> dict[str, torch.Tensor]:
    return {n: _value(n, tuple(s), seed) for n, s in named_shapes}


@torch.no_grad()
def init_deterministic_(model: torch.nn.Module, seed: int = 42) -> torch.nn.Module:
    """Overwrites every parameter of `model` (not buffers) with deterministic values."""
    for n, p in model.named_parameters():
        p.copy_(_value(n, tuple(p.shape), seed).to(p.device))
    return model
