"""B2TExperiment — mirrors reference src/experiments/b2t_experiment.py:17-111: the CTC character
tokenizer, the brain-to-text datasets and their loaders (optionally day-batched), greedy-decode
evaluation. The tokenizer is built offline (datasets/tokenizer.py). Without the .mat release
(yaml dataset_splits_dir absent) the experiment runs on the synthetic dataset of the same format
(`--synthetic_samples N`), which is what this container and the GPU box have."""
from __future__ import annotations

import os
from typing import Any, Literal, Optional

from torch.optim.optimizer import Optimizer
from torch.utils.data import DataLoader

from ..args.base_args import B2TDatasetArgsModel, BaseExperimentArgsModel
from ..datasets.brain2text import Brain2TextBatchSampler, Brain2TextDataset, SyntheticBrain2TextDataset
from ..datasets.tokenizer import create_ctc_tokenizer, vocab_of
from ..train.evaluator import DefaultEvaluator
from ..train.history import DecodedPredictionBatch
from .experiment import Experiment


class B2TArgsModel(BaseExperimentArgsModel, B2TDatasetArgsModel):
    tokenizer: Literal["wav2vec_pretrained", "ours"] = "wav2vec_pretrained"
    tokenizer_checkpoint: str = "facebook/wav2vec2-base-100h"
    day_batches: bool = False
    # build addition: synthetic trials when the .mat release is not present
    synthetic_samples: Optional[int] = None
    synthetic_min_len: int = 512
    synthetic_max_len: int = 1024


class B2TExperiment(Experiment):
    def __init__(self, config: dict, yamlConfig):
        self.config = self.get_args_model()(**config)
        self.yaml_config = yamlConfig
        self.tokenizer = self._create_tokenizer()
        super().__init__(config, yamlConfig)

    def get_name(self) -> str:
        raise NotImplementedError()

    @staticmethod
    def get_args_model():
        return B2TArgsModel

    def _create_tokenizer(self):
        if self.config.tokenizer == "wav2vec_pretrained":
            assert self.config.tokenizer_checkpoint is not None, \
                "Tokenizer checkpoint (--tokenizer_checkpoint) must be set when using --tokenizer=wav2vec_pretrained"
            return create_ctc_tokenizer(os.path.join(self.yaml_config.cache_dir, "tokenizer"))
        raise Exception(f"Tokenizer {self.config.tokenizer} not supported yet")

    def _create_model(self):
        raise NotImplementedError()

    def decode_predictions(self, predictions, sample) -> DecodedPredictionBatch:
        ids = predictions.logits.argmax(dim=-1).cpu().numpy()
        pred = self.tokenizer.batch_decode(ids, group_tokens=True)
        labels = (self.tokenizer.batch_decode(sample.target.cpu().numpy(), group_tokens=False)
                  if sample.target is not None else None)
        return DecodedPredictionBatch(pred, labels)

    def create_optimizer(self) -> Optimizer:
        cls: Any = self._get_optimizer_cls()
        return cls(self.model.parameters(), lr=self.config.learning_rate)

    def _use_synthetic(self) -> bool:
        d = getattr(self.yaml_config, "dataset_splits_dir", None)
        return self.config.synthetic_samples is not None or not d or not os.path.exists(d)

    def _create_dataset(self, split: Literal["train", "val", "test"] = "train"):
        if self._use_synthetic():
            n = self.config.synthetic_samples or 4 * self.config.batch_size
            seed = {"train": 0, "val": 1, "test": 2}[split] + 1000 * self.config.seed
            return SyntheticBrain2TextDataset(n if split == "train" else max(n // 4, 1), self.config.synthetic_min_len,
                                              self.config.synthetic_max_len, seed=seed, config=self.config)
        return Brain2TextDataset(config=self.config, yaml_config=self.yaml_config, split=split,
                                 tokenizer=self.tokenizer)

    def _create_dataloader(self, split: Literal["train", "val", "test"]) -> DataLoader:
        ds = self._create_dataset(split)
        collate = ds.get_collate_fn(self.tokenizer)
        if self.config.day_batches and split == "train" and self.world == 1:
            return DataLoader(ds, batch_sampler=Brain2TextBatchSampler(ds, self.base_config.batch_size),
                              collate_fn=collate)
        sampler = self._dp_sampler(ds, split)
        return DataLoader(ds, batch_size=self.base_config.batch_size, shuffle=split == "train" and sampler is None,
                          sampler=sampler, collate_fn=collate)

    def get_vocab(self) -> list[str]:
        return vocab_of(self.tokenizer)

    def create_evaluator(self, mode: Literal["train", "val", "test"], track_non_test_predictions: bool = False):
        return DefaultEvaluator(self.tokenizer, mode, track_non_test_predictions)
