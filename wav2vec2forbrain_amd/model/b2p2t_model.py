"""Day-dependent neural front end — mirrors reference src/model/b2p2t_model.py.

Forward (reference :138-179): permute -> GaussianSmoothing(k=20, 'same') -> per-sample day
linear (einsum btd,bdk) + day bias -> Softsign -> Unfold((32,1), stride 4) -> neural decoder.
Here smoothing + day linear + softsign run in functional.front_end (HIP), and the Unfold is an
implicit operand (functional.Unfolded) consumed by the GRU layer-0 projection GEMM: the
261 MB im2col tensor of the reference is never materialised.
"""
from __future__ import annotations

import math
from typing import Literal, cast

import torch
from pydantic import BaseModel
from torch import nn

from .. import functional as Fn
from ..datasets.batch_types import B2tSampleBatch
from .b2tmodel import B2TModel, ModelOutput

DEFAULT_UNFOLDER_KERNEL_LEN = 32


class B2P2TModelArgsModel(BaseModel):
    input_layer_nonlinearity: Literal["softsign"] = "softsign"
    unfolder_kernel_len: int = DEFAULT_UNFOLDER_KERNEL_LEN
    unfolder_stride_len: int = 4
    gaussian_smooth_width: float = 0.3


class GaussianSmoothing(nn.Module):
    """Depthwise Gaussian smoothing over time (reference :27-90). Keeps the reference buffer
    `weight` (channels, 1, kernel) for state_dict compatibility; the kernel itself is applied by
    the HIP front end."""

    def __init__(self, channels, kernel_size: int, sigma: float, dim=1):
        super().__init__()
        if dim != 1:
            raise NotImplementedError("only the 1-D smoothing used by B2P2TModel is supported")
        mgrid = torch.arange(kernel_size, dtype=torch.float32)
        mean = (kernel_size - 1) / 2
        kernel = 1 / (sigma * math.sqrt(2 * math.pi)) * torch.exp(-(((mgrid - mean) / sigma) ** 2) / 2)
        kernel = kernel / torch.sum(kernel)
        kernel = kernel.view(1, 1, kernel_size).repeat(channels, 1, 1)
        self.register_buffer("weight", kernel)
        self.groups = channels

    def taps(self) -> torch.Tensor:
        return self.weight[0, 0].contiguous()


class B2P2TModel(B2TModel):
    """Wraps the neural decoder model to perform trial day dependant preprocessing."""

    def __init__(self, config: B2P2TModelArgsModel, neural_decoder: B2TModel, pad_token_id=0):
        super().__init__()
        self.config = config
        self.pad_token_id = pad_token_id
        if config.input_layer_nonlinearity != "softsign":
            raise NotImplementedError("Only softsign is currently supported as input layer nonlinearity")
        n_days = 24
        neural_dim_len = 256
        self.gaussian_smoother = GaussianSmoothing(neural_dim_len, 20, config.gaussian_smooth_width, dim=1)
        self.day_weights = nn.Parameter(torch.randn(n_days, neural_dim_len, neural_dim_len))
        self.day_bias = nn.Parameter(torch.zeros(n_days, 1, neural_dim_len))
        for x in range(n_days):
            self.day_weights.data[x, :, :] = torch.eye(neural_dim_len)
        self.neural_decoder = neural_decoder
        # reference :129-136 — constructed but never used on the forward path; kept for state_dict parity
        for x in range(n_days):
            setattr(self, "inpLayer" + str(x), nn.Linear(neural_dim_len, neural_dim_len))
        for x in range(n_days):
            layer = getattr(self, "inpLayer" + str(x))
            layer.weight = nn.Parameter(layer.weight + torch.eye(neural_dim_len))

    def forward(self, batch: B2tSampleBatch) -> ModelOutput:
        x, targets = batch
        day_idxs = batch.day_idxs
        taps = self.gaussian_smoother.taps()
        s = Fn.front_end(x, day_idxs, self.day_weights, self.day_bias, taps)
        strided_inputs = Fn.Unfolded(s, self.config.unfolder_kernel_len, self.config.unfolder_stride_len)
        preprocessed_batch = batch.copy_and_change(input=strided_inputs)
        if hasattr(batch, "input_lens"):
            # ((input_lens - k) / stride).to(torch.int32), reference :170-173
            processed_in_lens = Fn.unfold_lens(batch.input_lens, self.config.unfolder_kernel_len,
                                               self.config.unfolder_stride_len)
            preprocessed_batch.input_lens = processed_in_lens
            out = self.neural_decoder.forward(preprocessed_batch)
            out.logit_lens = processed_in_lens
            return out
        return self.neural_decoder.forward(preprocessed_batch)

    def output_length(self, L: int) -> int:
        """Frames of the Unfold((k,1), stride) of L input bins (Fn.Unfolded.T): what the encoder sees."""
        return (L - self.config.unfolder_kernel_len) // self.config.unfolder_stride_len + 1

    @classmethod
    def get_in_size_after_preprocessing(cls, unfolder_kernel_len: int):
        return 256 * unfolder_kernel_len
