"""Evaluators — a minimal mirror of reference src/train/evaluator.py:20-120 (loss tracking, greedy
CTC decode, WER/CER). Train/val batches on the GPU get their word errors from the device decode
(functional.ctc_greedy_wer, csrc/decode.hip); the host path (test mode, CER, CPU
tensors) restates the reference's torcheval / edit_distance metrics, which are absent here."""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..model.b2tmodel import ModelOutput


def edit_distance(a, b) -> int:
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def greedy_ctc_decode(ids, vocab, blank=0, word_delimiter="|"):
    """argmax ids -> group repeats -> drop blank/pad -> string (tokenizer.batch_decode(group_tokens=True))."""
    out, last = [], None
    for i in ids:
        if i != last and i != blank:
            tok = vocab[i] if i < len(vocab) else ""
            if not (tok.startswith("<") and tok.endswith(">")):
                out.append(" " if tok == word_delimiter else tok)
        last = i
    return "".join(out).strip()


@dataclass
class EpochResult:
    losses: list = field(default_factory=list)
    metrics: dict = field(default_factory=dict)

    def get_average_loss(self):
        return sum(self.losses) / max(len(self.losses), 1)


class Evaluator:
    def __init__(self, mode: str, vocab=None, decode: bool = False):
        self.mode = mode
        self.vocab = vocab
        self.decode = decode and vocab is not None
        self.result = EpochResult()
        self.word_errs = self.words = self.char_errs = self.chars = 0

    def track_batch(self, predictions: ModelOutput, sample):
        loss = predictions.metrics.get("ctc_loss")
        if loss is None and predictions.loss is not None:
            loss = predictions.loss.item()
        if isinstance(loss, torch.Tensor):
            loss = loss.item()
        self.result.losses.append(float(loss))
        if self.decode and sample.target is not None and predictions.logits.is_cuda and self.mode != "test":
            # word errors on the device (csrc/decode.hip): no argmax / strings round trip per step;
            # the sums stay on the device until evaluate()
            from .. import functional as Fn
            ids = {t: i for i, t in enumerate(self.vocab)}
            _, errs, nw, _, _ = Fn.ctc_greedy_wer(predictions.logits.detach().contiguous(), sample.target,
                                                  blank=ids.get("<pad>", 0), eos=ids.get("</s>", 2),
                                                  delim=ids.get("|", 4))
            self.dev_errs = errs.sum() + getattr(self, "dev_errs", 0)
            self.dev_words = nw.sum() + getattr(self, "dev_words", 0)
            return
        if self.decode and sample.target is not None:
            pred = predictions.logits.argmax(-1).cpu().tolist()
            tgt = sample.target.cpu().tolist()
            for p, t in zip(pred, tgt):
                ps = greedy_ctc_decode(p, self.vocab)
                ts = greedy_ctc_decode([x for x in t if x > 0], self.vocab) if False else \
                    "".join(" " if self.vocab[x] == "|" else self.vocab[x] for x in t if x > 0).strip()
                self.word_errs += edit_distance(ps.split(), ts.split())
                self.words += max(len(ts.split()), 1)
                self.char_errs += edit_distance(ps, ts)
                self.chars += max(len(ts), 1)

    def get_latest_loss(self):
        return self.result.losses[-1]

    def get_running_loss(self):
        return self.result.get_average_loss()

    def evaluate(self) -> EpochResult:
        if getattr(self, "dev_words", None) is not None:
            self.result.metrics["word_error_rate"] = float(self.dev_errs) / max(float(self.dev_words), 1.0)
        if self.decode and self.words:
            self.result.metrics["word_error_rate"] = self.word_errs / self.words
            self.result.metrics["char_error_rate"] = self.char_errs / self.chars
        return self.result

    def clean_up(self):
        pass
