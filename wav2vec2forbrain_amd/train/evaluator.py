"""Evaluators — mirror reference src/train/evaluator.py:20-242 (per-batch loss, greedy CTC decode,
word and character error rates into a SingleEpochHistory).

The reference decodes every batch on the host (logits.argmax(-1).cpu() -> tokenizer.batch_decode ->
torcheval WordErrorRate / edit_distance CER). Here a batch whose logits are on the GPU gets its
word and character errors from the device decode kernels (csrc/decode.hip: functional.
ctc_greedy_wer / ctc_greedy_cer) and only the scalars cross to the host, in one
transfer with the loss. Strings are still built on the host where the reference keeps them (test
mode, track_non_test_predictions), from the same greedy decode.

LM decoding (pyctcdecode + KenLM through Wav2Vec2ProcessorWithLM, src/train/evaluator.py:148-210)
needs hub/KenLM assets that are not available offline; lm_decode_test_predictions raises.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from math import nan
from typing import Literal

import torch

from ..model.b2tmodel import ModelOutput
from .history import DecodedPredictionBatch, MetricEntry, SingleEpochHistory


def edit_distance(a, b) -> int:
    """Levenshtein distance (unit costs) between two sequences (host path)."""
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def cut_after_eos_token(s: str, eos: str = "</s>") -> str:
    i = s.find(eos)
    return s if i == -1 else s[:i + len(eos)]


def word_error_rate(preds: list[str], targets: list[str]) -> float:
    """torcheval WordErrorRate over a batch: summed word edit distances / summed target words."""
    errs = sum(edit_distance(p.split(), t.split()) for p, t in zip(preds, targets))
    n = sum(len(t.split()) for t in targets)
    return errs / n if n else nan


def char_error_rate(preds: list[str], targets: list[str]) -> float:
    """Reference calculate_char_error_rate: summed character edit distances / summed target lengths."""
    errs = sum(edit_distance(t, p) for p, t in zip(preds, targets))
    n = sum(len(t) for t in targets)
    return errs / n if n else nan


def _ids(tokenizer):
    v = tokenizer.get_vocab()
    return v.get(tokenizer.pad_token, 0), v.get(tokenizer.eos_token, 2), v.get(tokenizer.word_delimiter_token, 4)


class Evaluator(ABC):
    def __init__(self, mode: Literal["train", "val", "test"], track_non_test_predictions: bool = False):
        self.running_loss = 0.0
        self.n_losses = 0
        self.latest_loss = nan
        self.mode = mode
        self.track_non_test_predictions = track_non_test_predictions

    def track_batch(self, predictions: ModelOutput, sample):
        assert predictions.loss is not None
        loss = self._track_batch(predictions, sample)
        self.running_loss += loss
        self.n_losses += 1
        self.latest_loss = loss

    def get_running_loss(self):
        return self.running_loss / self.n_losses

    def get_latest_loss(self):
        return self.latest_loss

    @abstractmethod
    def _track_batch(self, predictions: ModelOutput, sample) -> float:
        """Records the batch; returns its loss as a float."""

    @abstractmethod
    def evaluate(self) -> SingleEpochHistory:
        raise NotImplementedError()

    def clean_up(self):
        pass


class DefaultEvaluator(Evaluator):
    """Greedy decode + word error rate per batch (reference :57-120)."""

    with_cer = False

    def __init__(self, tokenizer, mode: Literal["train", "val", "test"], track_non_test_predictions: bool = False):
        super().__init__(mode, track_non_test_predictions)
        self.history = SingleEpochHistory()
        self.tokenizer = tokenizer

    def keep_strings(self) -> bool:
        return self.mode == "test" or self.track_non_test_predictions

    def decode_predictions(self, predictions: ModelOutput, sample) -> DecodedPredictionBatch:
        ids = predictions.logits.argmax(dim=-1).cpu().numpy()
        pred = self.tokenizer.batch_decode(ids, group_tokens=True)
        labels = (self.tokenizer.batch_decode(sample.target.cpu().numpy(), group_tokens=False)
                  if sample.target is not None else None)
        return DecodedPredictionBatch(pred, labels)

    def _device_metrics(self, predictions: ModelOutput, sample) -> list[torch.Tensor]:
        from .. import functional as Fn
        from ..datasets.tokenizer import vocab_of
        blank, eos, delim = _ids(self.tokenizer)
        logits = predictions.logits.detach().contiguous()
        wer, _, nw, _, _ = Fn.ctc_greedy_wer(logits, sample.target, blank=blank, eos=eos, delim=delim)
        out = [torch.where(nw.sum() > 0, wer, torch.full_like(wer, nan))]
        if self.with_cer:
            cer, errs, nch = Fn.ctc_greedy_cer(logits, sample.target, vocab_of(self.tokenizer), blank=blank, eos=eos,
                                               delim=delim)
            out.append(torch.where(nch.sum() > 0, cer, torch.full_like(cer, nan)))
            out.append((errs < 0).sum())   # rows the device decode could not hold: scored on the host
        return out

    def _track_batch(self, predictions: ModelOutput, sample) -> float:
        loss_t = predictions.loss.detach().reshape(())
        decoded = None
        extra = {}
        if sample.target is not None and predictions.logits.is_cuda and not self.keep_strings():
            vals = torch.stack([loss_t.float()] + [v.float().to(loss_t.device) for v in
                                                   self._device_metrics(predictions, sample)]).tolist()
            loss = vals[0]
            extra["word_error_rate"] = vals[1]
            if self.with_cer:
                extra["char_error_rate"] = vals[2]
                if vals[3] > 0:   # a decoded string overflowed the device buffer: the host path
                    pred, labels = self.decode_predictions(predictions, sample)
                    extra["char_error_rate"] = char_error_rate([cut_after_eos_token(x) for x in pred], labels)
        else:
            loss = float(loss_t)
            pred, labels = self.decode_predictions(predictions, sample)
            pred = [cut_after_eos_token(s) for s in pred]
            if labels is not None:
                extra["word_error_rate"] = word_error_rate(pred, labels)
                if self.with_cer:
                    extra["char_error_rate"] = char_error_rate(pred, labels)
            decoded = DecodedPredictionBatch(pred, labels) if self.keep_strings() else None
        metrics = {k: (float(v) if isinstance(v, torch.Tensor) else v) for k, v in predictions.metrics.items()}
        metrics.update(extra)
        predictions.metrics.update(extra)
        self.history.add_batch_metric(MetricEntry(metrics, loss), decoded)
        return loss

    def evaluate(self) -> SingleEpochHistory:
        return self.history


class EvaluatorWithW2vLMDecoder(DefaultEvaluator):
    """DefaultEvaluator + character error rate (reference :127-242)."""

    with_cer = True

    def __init__(self, tokenizer, mode: Literal["train", "val", "test"], cache_dir: str = "",
                 processor_checkpoint: str = "", track_non_test_predictions: bool = False,
                 lm_decode_test_predictions: bool = False, lm_decode_beam_width=None, lm_decode_beam_prune_logp=None,
                 lm_decode_token_min_logp=None, lm_decode_alpha=None, lm_decode_beta=None,
                 lm_decode_score_boundary=None, beam_decode_test_predictions: bool = False):
        super().__init__(tokenizer, mode, track_non_test_predictions)
        # LM-free CTC prefix beam search on the device (csrc/beam.hip) with the LM decode's beam width /
        # pruning: test-mode metrics word/char_error_rate_beam_decode (the LM decode needs hub assets)
        self.beam_decode = bool(beam_decode_test_predictions)
        self.beam_cfg = dict(beam=lm_decode_beam_width or 100,
                             beam_prune_logp=-10.0 if lm_decode_beam_prune_logp is None else lm_decode_beam_prune_logp,
                             token_min_logp=-5.0 if lm_decode_token_min_logp is None else lm_decode_token_min_logp)
        if lm_decode_test_predictions and mode == "test":
            raise NotImplementedError(
                f"LM decoding needs Wav2Vec2ProcessorWithLM.from_pretrained({processor_checkpoint!r}) and its KenLM "
                "model, which are not available offline")
        self.lm_decode_beam_width = lm_decode_beam_width
        self.lm_decode_alpha, self.lm_decode_beta = lm_decode_alpha, lm_decode_beta

    def beam_decode_predictions(self, predictions: ModelOutput) -> list[str]:
        """Best prefixes of the device beam search as strings (cut after </s>, like the greedy path)."""
        from .. import functional as Fn
        blank, _, _ = _ids(self.tokenizer)
        tok, n, _ = Fn.ctc_prefix_beam(predictions.logits.detach().float().contiguous(), predictions.logit_lens,
                                       blank=blank, **self.beam_cfg)
        tok, n = tok.cpu().numpy(), n.cpu().numpy()
        return [cut_after_eos_token(self.tokenizer.decode(list(tok[b, :n[b]]), group_tokens=False))
                for b in range(tok.shape[0])]

    def _track_batch(self, predictions: ModelOutput, sample) -> float:
        if self.beam_decode and self.mode == "test" and sample.target is not None and predictions.logits.is_cuda:
            labels = self.tokenizer.batch_decode(sample.target.cpu().numpy(), group_tokens=False)
            pred = self.beam_decode_predictions(predictions)
            predictions.metrics.update({"word_error_rate_beam_decode": word_error_rate(pred, labels),
                                        "char_error_rate_beam_decode": char_error_rate(pred, labels)})
        return super()._track_batch(predictions, sample)
