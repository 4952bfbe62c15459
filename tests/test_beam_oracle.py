"""Known-answer check of the CTC prefix beam search restatement (oracle/ctc_beam_oracle.py), CPU:
with an unbounded beam and no pruning the prefix beam search is exact, so its best prefix and log
probability must equal a brute-force sum over every alignment (T^C paths) of tiny cases."""
import itertools
import math

import numpy as np
import pytest

from oracle.ctc_beam_oracle import ctc_prefix_beam, log_softmax32


def _brute(logits, blank=0):
    T, C = logits.shape
    y = np.stack([log_softmax32(logits[t]) for t in range(T)]).astype(np.float64)
    probs = {}
    for path in itertools.product(range(C), repeat=T):
        lp = sum(y[t, c] for t, c in enumerate(path))
        col = tuple(c for i, c in enumerate(path) if (i == 0 or c != path[i - 1]) and c != blank)
        probs[col] = np.logaddexp(probs.get(col, -np.inf), lp)
    best = max(probs, key=probs.get)
    return best, probs[best]


@pytest.mark.parametrize("seed", range(6))
def test_unbounded_beam_is_exact(seed):
    rng = np.random.default_rng(seed)
    T, C = 6, 3
    logits = (rng.standard_normal((T, C)) * 2.0).astype(np.float32)
    pre, lp = ctc_prefix_beam(logits, beam=10 ** 6, token_min_logp=-math.inf, beam_prune_logp=-math.inf)
    bpre, blp = _brute(logits)
    assert pre == bpre
    assert abs(float(lp) - blp) < 1e-4


def test_empty_and_single_frame():
    assert ctc_prefix_beam(np.zeros((0, 4), np.float32), 4) == ((), 0.0)
    pre, _ = ctc_prefix_beam(np.array([[0.0, 5.0, 0.0]], np.float32), 4)
    assert pre == (1,)
