"""Brain-to-text data: the .mat session files of the Willett et al. speech-BCI release, the block
z-scoring, the collate function that builds B2tSampleBatch, the day-batched sampler, and a synthetic
dataset of the same format.

Host-side by design: this runs once per dataset load / per batch on the CPU (DataLoader workers),
off the training step's hot path. Restated from the reference:
  session loading + split by block        src/datasets/brain2text.py:79-145
  feature preprocessing (z-score per block) src/datasets/preprocessing.py:30-216
  resampling                              src/datasets/preprocessing.py:12-27
  collate (zero-pad, tokenize, lengths)    src/datasets/brain2text.py:161-213
  day-batched sampler                      src/util/batch_sampler.py:8-55
"""
from __future__ import annotations

import os
import random
import re
from pathlib import Path
from typing import Callable, Literal, NamedTuple, Optional

import numpy as np
import torch
from torch.utils.data import Dataset, Sampler

from ..util.nn_helper import calc_seq_len
from .batch_types import B2tSampleBatch

# the 24 recording sessions, sorted: the day index of a sample is its session's position
SESSION_NAMES = sorted([
    "t12.2022.04.28", "t12.2022.05.05", "t12.2022.05.17", "t12.2022.05.19", "t12.2022.05.24", "t12.2022.05.26",
    "t12.2022.06.02", "t12.2022.06.07", "t12.2022.06.14", "t12.2022.06.16", "t12.2022.06.21", "t12.2022.06.23",
    "t12.2022.06.28", "t12.2022.07.05", "t12.2022.07.14", "t12.2022.07.21", "t12.2022.07.27", "t12.2022.07.29",
    "t12.2022.08.02", "t12.2022.08.11", "t12.2022.08.13", "t12.2022.08.18", "t12.2022.08.23", "t12.2022.08.25",
])

Area = Literal["44", "6v"]


class Sample(NamedTuple):
    input: torch.Tensor
    target: object


class B2tSample(Sample):
    day_idx: int


# ------------------------------------------------------------------------------ preprocessing
def _area_cols(area: Area) -> slice:
    # electrode array columns: the first 128 are area 6v, the last 128 area 44
    return slice(128, None) if area == "44" else slice(None, 128)


def _trial_feature(data_file: dict, name: str, i: int, area: Area) -> np.ndarray:
    return np.asarray(data_file[name][0, i])[:, _area_cols(area)]


def _sentences(data_file: dict) -> list[str]:
    return [str(s).strip() for s in np.asarray(data_file["sentenceText"]).reshape(-1)]


def _zscore_blocks(per_trial: list[np.ndarray], blocks: list[np.ndarray], texts: list[str], apply: bool):
    """Mean/std over all frames of a block's trials (contiguous trial index range), per feature."""
    feats, outs = [], []
    for idx in blocks:
        if apply:
            frames = np.concatenate(per_trial[idx[0]:idx[-1] + 1], axis=0)
            mu = frames.mean(axis=0, keepdims=True)
            sd = frames.std(axis=0, keepdims=True)
        for i in idx:
            feats.append((per_trial[i] - mu) / (sd + 1e-8) if apply else per_trial[i])
            outs.append(texts[i])
    return feats, outs


def _single(name: str, zscore: bool):
    def fn(data_file: dict, blocks: list[np.ndarray], area: Area):
        texts = _sentences(data_file)
        per_trial = [_trial_feature(data_file, name, i, area) for i in range(len(texts))]
        return _zscore_blocks(per_trial, blocks, texts, zscore)
    return fn


def preprocess_competition_recommended(data_file: dict, blocks: list[np.ndarray], area: Area):
    """[tx1 | spikePow] concatenated, then one z-score over the 256 columns per block."""
    texts = _sentences(data_file)
    per_trial = [np.concatenate([_trial_feature(data_file, "tx1", i, area),
                                 _trial_feature(data_file, "spikePow", i, area)], axis=1) for i in range(len(texts))]
    return _zscore_blocks(per_trial, blocks, texts, True)


def _separate(layout: str):
    def fn(data_file: dict, blocks: list[np.ndarray], area: Area):
        tx, texts = _single("tx1", True)(data_file, blocks, area)
        sp, _ = _single("spikePow", True)(data_file, blocks, area)
        if layout == "concat":      # (T, 256): tx then spike power, each z-scored on its own
            return [np.concatenate([a, b], axis=1) for a, b in zip(tx, sp)], texts
        if layout == "2ch":         # (2, T, 128)
            return [np.stack([a, b], axis=0) for a, b in zip(tx, sp)], texts
        return [np.stack([a[:, :64], a[:, 64:], b[:, :64], b[:, 64:]], axis=0) for a, b in zip(tx, sp)], texts
    return fn


PREPROCESSING: dict[str, Callable] = {
    "competition_recommended": preprocess_competition_recommended,
    "seperate_zscoring": _separate("concat"),
    "only_tx_unnormalized": _single("tx1", False),
    "only_tx_zscored": _single("tx1", True),
    "only_spikepow_unnormalized": _single("spikePow", False),
    "only_spikepow_zscored": _single("spikePow", True),
    "seperate_zscoring_2channels": _separate("2ch"),
    "seperate_zscoring_4channels": _separate("4ch"),
}


def resample_sample(sample: torch.Tensor, target_sample_rate: int, orig_sample_rate: int) -> torch.Tensor:
    """Linear time interpolation by the integer factor target // orig (frames x features)."""
    if target_sample_rate == orig_sample_rate:
        return sample
    f = target_sample_rate // orig_sample_rate
    x = sample.t().unsqueeze(0)
    return torch.nn.functional.interpolate(x, scale_factor=f, mode="linear").squeeze(0).t()


def block_ranges(block_idx: np.ndarray, split: str, competition_mode: bool) -> list[np.ndarray]:
    """Trial index sets per recording block; without competition mode the first block of each
    session is held out as the test split and the train split takes the remaining blocks."""
    nums = np.squeeze(block_idx)
    ids = list(np.unique(nums))
    if not competition_mode:
        if split == "test":
            ids = ids[:1]
        elif split == "train":
            ids = ids[1:]
    return [np.argwhere(nums == b)[:, 0].astype(np.int32) for b in ids]


# ------------------------------------------------------------------------------ datasets
class Brain2TextDataset(Dataset):
    """One sample per trial: (frames, 256) z-scored features, its uppercased sentence and the day
    index of its session. Split directories under yaml_config.dataset_splits_dir: train/, test/
    (also the validation split) and competitionHoldOut/."""

    def __init__(self, config, yaml_config, split: Literal["train", "val", "test"] = "train", tokenizer=None):
        from scipy.io import loadmat
        self.config = config
        self.tokenizer = tokenizer
        root = Path(yaml_config.dataset_splits_dir)
        sub = "test" if split == "val" else ("competitionHoldOut" if split == "test" and config.competition_mode
                                             else "train")
        path = root / sub
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} does not exist.")
        pre = PREPROCESSING[config.preprocessing]
        self.samples: list[B2tSample] = []
        for day, name in enumerate(SESSION_NAMES):
            f = path / f"{name}.mat"
            if not os.path.exists(f):
                continue
            data = loadmat(f)
            blocks = block_ranges(data["blockIdx"], split, config.competition_mode)
            feats, texts = pre(data, blocks, config.area)
            if len(feats) != len(texts):
                raise ValueError("features and transcriptions differ in length")
            for x, t in zip(feats, texts):
                s = B2tSample(torch.tensor(x, dtype=torch.float32), t.upper())
                s.day_idx = day
                self.samples.append(s)

    def __len__(self):
        n = len(self.samples)
        return n if self.config.limit_samples is None else min(n, self.config.limit_samples)

    def __getitem__(self, index: int) -> B2tSample:
        s = self.samples[index]
        x = resample_sample(s.input, self.config.sample_rate, 50)
        out = B2tSample(x, s.target)
        out.day_idx = s.day_idx
        return out

    def get_collate_fn(self, tokenizer=None):
        return make_collate_fn(tokenizer or self.tokenizer, self.config)


def make_collate_fn(tokenizer, config) -> Callable[[list[B2tSample]], B2tSampleBatch]:
    """Zero-pad the frames to the longest trial, tokenize the (punctuation-stripped) sentences with
    longest padding (pad id 0), day_idxs, input_lens = unpadded frame counts, target_lens = last
    non-pad index + 1 (calc_seq_len)."""
    if tokenizer is None:
        raise ValueError("Tokenizer must be provided for this implementation of collate function.")
    multi = config.preprocessing in ("seperate_zscoring_2channels", "seperate_zscoring_4channels")
    tdim = 1 if multi else 0
    strip = re.compile(r'[\,\?\.\!\-\;\:"]')

    def collate(batch: list[B2tSample]) -> B2tSampleBatch:
        T = max(x.size(tdim) for x, _ in batch)
        xs = [torch.nn.functional.pad(x, (0, 0, 0, T - x.size(tdim))) for x, _ in batch]
        texts = [strip.sub("", t) if config.remove_punctuation else t for _, t in batch]
        ids = tokenizer(texts, padding="longest", return_tensors="pt").input_ids
        out = B2tSampleBatch(torch.stack(xs), ids)
        out.day_idxs = torch.tensor([s.day_idx for s in batch])
        out.input_lens = torch.tensor([x.size(0) for x, _ in batch])
        out.target_lens = torch.tensor([calc_seq_len(r) for r in ids])
        return out

    return collate


class SyntheticBrain2TextDataset(Dataset):
    """Synthetic trials of the real format: x ~ N(0,1) (frames, 256) with frame
    counts in [min_len, max_len], random uppercase sentences over the CTC vocabulary's letters,
    day ~ U{0..23}. Deterministic from `seed`; used where the .mat release is absent (this
    container, the bench, the experiment tests)."""

    LETTERS = "ETAONIHSRDLUMWCFGYPBVKXJQZ'"

    def __init__(self, n: int, min_len: int = 512, max_len: int = 1024, seed: int = 0, words=(4, 12),
                 config=None):
        g = torch.Generator().manual_seed(seed)
        self.config = config
        self.samples: list[B2tSample] = []
        for _ in range(n):
            T = int(torch.randint(min_len, max_len + 1, (1,), generator=g))
            x = torch.randn(T, 256, generator=g)
            nw = int(torch.randint(words[0], words[1] + 1, (1,), generator=g))
            ws = []
            for _ in range(nw):
                k = int(torch.randint(2, 8, (1,), generator=g))
                ws.append("".join(self.LETTERS[int(i)] for i in torch.randint(0, len(self.LETTERS), (k,), generator=g)))
            s = B2tSample(x, " ".join(ws))
            s.day_idx = int(torch.randint(0, 24, (1,), generator=g))
            self.samples.append(s)

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        return self.samples[index]

    def get_collate_fn(self, tokenizer):
        class _Cfg:
            preprocessing = "seperate_zscoring"
            remove_punctuation = True
        return make_collate_fn(tokenizer, self.config or _Cfg)


class Brain2TextBatchSampler(Sampler):
    """Batches drawn within one session (day) at a time, shuffled; the last batch of a day may be
    short (reference src/util/batch_sampler.py:8-55)."""

    def __init__(self, data, batch_size: int, shuffle: bool = True):
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.by_day: dict[int, list[int]] = {}
        for i, s in enumerate(data.samples):
            self.by_day.setdefault(s.day_idx, []).append(i)
        self.batches = self._build()

    def _build(self) -> list[list[int]]:
        out = []
        for idx in self.by_day.values():
            random.shuffle(idx)
            for k in range(0, len(idx), self.batch_size):
                out.append(idx[k:k + self.batch_size])
        return out

    def __iter__(self):
        if self.shuffle:
            random.shuffle(self.batches)
        yield from self.batches

    def __len__(self):
        return len(self.batches)
