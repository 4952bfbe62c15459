"""Mirrors reference src/util/nn_helper.py:31-57 (create_fully_connected, calc_seq_len)."""
from __future__ import annotations

from typing import Literal

import torch
from torch import nn
from torch.nn import Linear

ACTIVATION_FUNCTION = Literal["gelu", "gelu_10", "gelu_fast", "gelu_new", "gelu_python", "gelu_pytorch_tanh",
                              "gelu_accurate", "laplace", "linear", "mish", "quick_gelu", "relu", "relu2", "relu6",
                              "sigmoid", "silu", "swish", "tanh"]

# activations with a fused HIP epilogue (GEMM act / act_bwd)
SUPPORTED_ACTIVATIONS = {"gelu": "gelu", "gelu_python": "gelu", "silu": "silu", "swish": "silu"}


class Activation(nn.Module):
    """Parameter-free marker for an activation between two Linear layers (fused into the GEMM)."""

    def __init__(self, name: str):
        super().__init__()
        if name not in SUPPORTED_ACTIVATIONS:
            raise NotImplementedError(f"activation {name!r} has no fused HIP epilogue; supported: "
                                      f"{sorted(SUPPORTED_ACTIVATIONS)}")
        self.name = SUPPORTED_ACTIVATIONS[name]

    def forward(self, x):  # pragma: no cover - fused by the caller
        raise RuntimeError("Activation is fused into the preceding Linear")


def create_fully_connected(input_size: int, output_size: int, hidden_sizes=[], activation="gelu",
                           use_batch_norm: bool = False):
    if use_batch_norm:
        raise NotImplementedError("use_batch_norm is not used on the b2p2t_gru+w2v path")
    layers = []
    for i in range(-1, len(hidden_sizes)):
        is_last = i + 1 == len(hidden_sizes)
        is_first = i == -1
        in_size = input_size if is_first else hidden_sizes[i]
        out_size = output_size if is_last else hidden_sizes[i + 1]
        layers.append(Linear(in_size, out_size))
        if not is_last:
            layers.append(Activation(activation))
    return nn.Sequential(*layers)


def run_fully_connected(seq: nn.Sequential, x):
    """Applies a create_fully_connected stack with each activation fused into its Linear."""
    from .. import functional as Fn
    mods = list(seq)
    i = 0
    while i < len(mods):
        lin = mods[i]
        act = 0
        if i + 1 < len(mods) and isinstance(mods[i + 1], Activation):
            act = Fn.ACT[mods[i + 1].name]
            i += 1
        x = Fn.linear(x, lin.weight, lin.bias, act)
        i += 1
    return x


def calc_seq_len(index_seq: torch.Tensor):
    for i in range(len(index_seq)):
        j = len(index_seq) - 1 - i
        if index_seq[j].item() > 0:
            return j + 1
    return 0
