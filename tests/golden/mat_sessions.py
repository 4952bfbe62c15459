"""Synthetic session files in the format of the speech-BCI release (.mat per session: tx1 and
spikePow as 1 x n_trials cells of (frames, 256) matrices, sentenceText, blockIdx), deterministic
from a seed. Shared by make_golden_data.py (reference side) and tests/test_data_pipeline.py."""
from __future__ import annotations

import os

import numpy as np

SESSIONS = {"t12.2022.05.05": 11, "t12.2022.07.21": 12}   # name -> seed (two days: day indices 1 and 15)
WORDS = ["the", "quick", "brown", "fox", "jumps", "over", "a", "lazy", "dog", "it's", "here", "now"]


def session_arrays(seed: int) -> dict:
    rng = np.random.default_rng(seed)
    blocks = [int(b) for b in rng.integers(2, 4, size=3)]      # trials per block
    n = sum(blocks)
    tx, sp, text = [], [], []
    for _ in range(n):
        T = int(rng.integers(20, 41))
        tx.append(rng.poisson(2.0, size=(T, 256)).astype(np.float64))
        sp.append(rng.gamma(2.0, 30.0, size=(T, 256)))
        k = int(rng.integers(2, 6))
        s = " ".join(rng.choice(WORDS, size=k)) + rng.choice([".", "?", "", "!"])
        text.append(s + "   ")      # char-matrix padding, stripped on load
    cell_tx = np.empty((1, n), dtype=object)
    cell_sp = np.empty((1, n), dtype=object)
    for i in range(n):
        cell_tx[0, i] = tx[i]
        cell_sp[0, i] = sp[i]
    block_idx = np.concatenate([np.full(b, j + 1) for j, b in enumerate(blocks)]).reshape(-1, 1)
    return {"tx1": cell_tx, "spikePow": cell_sp, "sentenceText": np.array(text), "blockIdx": block_idx}


def write_splits(root: str) -> str:
    """root/{train,test}/<session>.mat (the same files in both, as the release's layout)."""
    from scipy.io import savemat
    for split in ("train", "test"):
        os.makedirs(os.path.join(root, split), exist_ok=True)
        for name, seed in SESSIONS.items():
            savemat(os.path.join(root, split, f"{name}.mat"), session_arrays(seed))
    return root
