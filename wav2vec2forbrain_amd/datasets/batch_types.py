"""Batch containers — mirrors reference src/datasets/batch_types.py:5-41 (NamedTuple with dynamic
attributes moved to the device by .cuda(); copy_and_change keeps them)."""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch


class SampleBatch(NamedTuple):
    input: torch.Tensor
    target: Optional[torch.Tensor]

    def cuda(self):
        copy = self._replace(
            input=self.input.cuda(non_blocking=True),
            target=self.target.cuda(non_blocking=True) if self.target is not None else None,
        )
        if hasattr(self, "__dict__"):
            for key, value in self.__dict__.items():
                if isinstance(value, torch.Tensor):
                    copy.__setattr__(key, value.cuda(non_blocking=True))
                else:
                    copy.__setattr__(key, value)
        return copy

    def copy_and_change(self, **diff):
        copy = self._replace(**diff)
        for key, value in self.__dict__.items():
            copy.__setattr__(key, value)
        return copy


class B2tSampleBatch(SampleBatch):
    day_idxs: torch.Tensor
    input_lens: torch.Tensor
    target_lens: Optional[torch.Tensor]


class PhonemeSampleBatch(B2tSampleBatch):
    transcriptions: Optional[list[str]]
    phonemes: list[list[str]]


def make_b2t_batch(x, target, day_idxs, input_lens, target_lens) -> B2tSampleBatch:
    b = B2tSampleBatch(x, target)
    b.day_idxs = day_idxs
    b.input_lens = input_lens
    b.target_lens = target_lens
    return b
