"""Model I/O types — mirrors reference src/model/b2tmodel.py:9-21."""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Optional

import torch
from torch.nn import Module

from ..datasets.batch_types import SampleBatch


@dataclass
class ModelOutput:
    logits: torch.Tensor
    metrics: dict[str, float]
    loss: Optional[torch.Tensor] = None
    logit_lens: Optional[torch.Tensor] = None
    hidden_states: Optional[torch.Tensor] = None


class B2TModel(Module, ABC):
    @abstractmethod
    def forward(self, batch: SampleBatch) -> ModelOutput:
        pass
