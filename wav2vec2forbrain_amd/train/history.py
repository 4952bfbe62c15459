"""Training history records — the reference's result format (src/train/history.py:6-180), so that
history.json files and checkpoint-resume histories are interchangeable between the two."""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from math import nan
from typing import NamedTuple, Optional


class DecodedPredictionBatch(NamedTuple):
    predictions: list[str]
    targets: Optional[list[str]]


@dataclass
class MetricEntry:
    metrics: dict = field(default_factory=dict)
    loss: float = 0.0

    def __iadd__(self, other: "MetricEntry"):
        for k, v in other.metrics.items():
            self.metrics[k] = self.metrics[k] + v if self.metrics.get(k) is not None else v
        self.loss += other.loss
        return self

    def __truediv__(self, n: float):
        if n == 0:
            return MetricEntry({k: nan for k in self.metrics}, nan)
        return MetricEntry({k: v / n for k, v in self.metrics.items()}, self.loss / n)


class SingleEpochHistory:
    def __init__(self):
        self.metrics: list[MetricEntry] = []
        self._total = MetricEntry({})
        self._count = 0
        self.decoded: list[Optional[DecodedPredictionBatch]] = []

    def add_batch_metric(self, entry: MetricEntry, decoded: Optional[DecodedPredictionBatch] = None):
        self.metrics.append(entry)
        self._total += MetricEntry(dict(entry.metrics), entry.loss)
        self._count += 1
        self.decoded.append(decoded)

    def get_average(self) -> MetricEntry:
        return self._total / self._count

    def get_last(self) -> MetricEntry:
        return self.metrics[-1]

    def to_dict(self):
        def batch(i):
            d = self.decoded[i]
            if d is None:
                return {}
            out = dict(d._asdict())
            out.update({k: v for k, v in getattr(d, "__dict__", {}).items()})
            return out
        return {"history": [{"metrics": m.metrics, "loss": m.loss, "batch": batch(i)} for i, m in enumerate(self.metrics)],
                "average": vars(self.get_average()) if self._count else {"metrics": {}, "loss": nan}}

    def plot_metric_as_hist(self, metric_key: str, title: str, ax):
        vals = [m.metrics[metric_key] for m in self.metrics if metric_key in m.metrics]
        ax.hist(vals, bins=10, color="blue", alpha=0.7)
        missing = len(self.metrics) - len(vals)
        ax.set_title(title + (f" (ignored {missing} batches w/o {metric_key})" if missing else ""))
        ax.set_xlabel(metric_key)
        ax.set_ylabel("Frequency")


class EpochLosses(NamedTuple):
    train_losses: SingleEpochHistory
    val_losses: SingleEpochHistory

    def to_dict(self):
        return {"train": self.train_losses.to_dict(), "val": self.val_losses.to_dict()}


def _history_from(d: dict) -> SingleEpochHistory:
    h = SingleEpochHistory()
    for b in d["history"]:
        dec = None
        if isinstance(b.get("batch"), dict) and "predictions" in b["batch"]:
            dec = DecodedPredictionBatch(b["batch"]["predictions"], b["batch"].get("targets"))
        h.add_batch_metric(MetricEntry(b["metrics"], b["loss"]), dec)
    return h


class TrainHistory(NamedTuple):
    epochs: list[EpochLosses]
    test_losses: SingleEpochHistory

    def to_dict(self):
        return {"epochs": [e.to_dict() for e in self.epochs], "test": self.test_losses.to_dict()}

    @classmethod
    def from_json(cls, path: str) -> "TrainHistory":
        with open(path) as f:
            data = json.load(f)
        epochs = [EpochLosses(_history_from(e["train"]), _history_from(e["val"])) for e in data["epochs"]]
        return cls(epochs, _history_from(data["test"]))

    def plot(self, out_path: str):
        if not self.epochs:
            return
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        keys = set()
        for e in self.epochs:
            keys |= set(e.train_losses.get_average().metrics) | set(e.val_losses.get_average().metrics)
        keys = sorted(keys)
        if not keys:
            return
        fig, axs = plt.subplots(nrows=len(keys), ncols=1, figsize=(10, 5 * len(keys)))
        for i, k in enumerate(keys):
            ax = axs[i] if len(keys) > 1 else axs
            tr = [e.train_losses.get_average().metrics.get(k) for e in self.epochs]
            va = [e.val_losses.get_average().metrics.get(k) for e in self.epochs]
            ax.plot([v for v in tr if v is not None], label=f"{k} (train)", marker="o")
            ax.plot([v for v in va if v is not None], label=f"{k} (validation)", marker=".")
            ax.grid()
            ax.set_xlabel("Epochs")
            ax.set_ylabel(k)
            ax.legend()
        plt.tight_layout()
        plt.savefig(out_path)
        plt.close(fig)
