"""TEST INFRASTRUCTURE ONLY — CPU restatement (numpy float32) of the LM-free CTC prefix beam search
that csrc/beam.hip runs on the device: the decoding the reference's test evaluator does with
pyctcdecode (src/train/evaluator.py:148-154,189-210) minus the KenLM language model, whose assets
are unavailable offline. pyctcdecode 0.5.0 (the reference environment's pin) is not installed here:
this restates its LM-free core, the prefix beam search of Hannun et al. (2014), with its two pruning
rules (token_min_logp: characters below it are skipped unless they are the frame's argmax;
beam_prune_logp: candidates below best + it are dropped). Parity of the kernel is pinned against
this restatement only ("parity unpinned" against pyctcdecode itself: no reference vectors exist).

Candidate order, merging and tie-breaking follow the kernel exactly: beam w (sorted position) and
character c give candidate k = w*C + c; the blank slot is beam w's "stay" candidate; an extension
l + c equal to a live beam's prefix is merged into that beam's stay candidate; the W best by
(descending log p, ascending k) survive."""
from __future__ import annotations

import numpy as np

NEG = np.float32(-np.inf)


def _lse(a, b):
    a, b = np.float32(a), np.float32(b)
    if a == NEG:
        return b
    if b == NEG:
        return a
    m = max(a, b)
    return np.float32(m + np.log1p(np.exp(np.float32(-abs(a - b)))))


def log_softmax32(v):
    v = np.asarray(v, np.float32)
    m = v.max()
    s = np.exp(v - m).sum(dtype=np.float32)
    return (v - m - np.log(s)).astype(np.float32)


def ctc_prefix_beam(logits, beam, blank=0, token_min_logp=-5.0, beam_prune_logp=-10.0, length=None):
    """logits (T, C) raw scores of one sample -> (token tuple of the best prefix, its log p)."""
    logits = np.asarray(logits, np.float32)
    T, C = logits.shape
    T = T if length is None else min(length, T)
    tmin = np.float32(token_min_logp)
    beams = [((), np.float32(0.0), NEG)]          # (prefix, log p_b, log p_nb), sorted slots
    for t in range(T):
        y = log_softmax32(logits[t])
        arg = int(np.argmax(y))
        use = [bool(y[c] >= tmin or c == arg) for c in range(C)]
        cand = {}
        for w, (pre, pb, pnb) in enumerate(beams):
            tot = _lse(pb, pnb)
            if tot == NEG:
                continue
            last = pre[-1] if pre else -1
            for c in range(C):
                vb, vnb = NEG, NEG
                if c == blank:
                    if use[c]:
                        vb = np.float32(tot + y[blank])
                    if last >= 0 and use[last]:
                        vnb = np.float32(pnb + y[last])
                elif use[c]:
                    vnb = np.float32((pb if c == last else tot) + y[c])
                cand[w * C + c] = [vb, vnb]
        # merge extensions that reproduce a live prefix into that beam's stay candidate
        index = {pre: w for w, (pre, pb, pnb) in enumerate(beams) if _lse(pb, pnb) != NEG}
        merged = []
        for w, (pre, pb, pnb) in enumerate(beams):
            if not pre or _lse(pb, pnb) == NEG or not use[pre[-1]]:
                continue
            w0 = index.get(pre[:-1])
            if w0 is None or w0 == w:
                continue
            ke = w0 * C + pre[-1]
            cand[w * C + blank][1] = _lse(cand[w * C + blank][1], cand[ke][1])
            merged.append(ke)
        for ke in merged:
            cand[ke] = [NEG, NEG]
        tots = {k: _lse(vb, vnb) for k, (vb, vnb) in cand.items()}
        best = max(tots.values()) if tots else NEG
        thr = np.float32(best + np.float32(beam_prune_logp))
        keep = sorted((k for k, v in tots.items() if v != NEG and v >= thr), key=lambda k: (-tots[k], k))[:beam]
        nb = []
        for k in keep:
            w, c = divmod(k, C)
            pre = beams[w][0]
            nb.append((pre if c == blank else pre + (c,), cand[k][0], cand[k][1]))
        beams = nb
    if not beams or T == 0:
        return (), np.float32(0.0)
    return beams[0][0], _lse(beams[0][1], beams[0][2])
