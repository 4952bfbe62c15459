"""Experiment base class — mirrors reference src/experiments/experiment.py:31-364 (the object
run.py builds and runs: seeds, data loaders, results directory, model construction and checkpoint
loading, optimizer / scheduler hooks, Trainer, prediction, stored artefacts).

Differences, all offline / platform consequences:
  * W&B logging: use_wandb=True raises (no network); results go to results_dir only.
  * prefix beam search with a causal LM (use_prefix_beam_search loads GPT-2 from the hub at
    construction, :87-95) is not loaded: the hub is unreachable and nothing on the training path
    uses it.
  * data-parallel runs (torchrun, one process per GPU): the train loader is sharded with a
    DistributedSampler (reshuffled every epoch by the Trainer's set_epoch), the dropout seed stream
    is offset by the rank (host torch seed equal on all ranks), rank 0 writes results.
  * the model's training step runs on the HIP kernels (functional.py); the optimizer is the
    multi-tensor HIP Adam (optim.HipAdam) with the reference's arguments (SGD stays torch's).
"""
from __future__ import annotations

import json
import os
import sys
from abc import ABCMeta, abstractmethod
from datetime import datetime
from typing import Any, Callable, Literal, Optional, Type, cast

import numpy as np
import torch
import torch.distributed as dist
from torch.optim.optimizer import Optimizer
from torch.utils.data import DataLoader

from ..args.base_args import BaseExperimentArgsModel
from ..datasets.batch_types import SampleBatch
from ..model.b2tmodel import B2TModel, ModelOutput
from ..train.history import SingleEpochHistory, TrainHistory


def _optimizers() -> dict[str, type]:
    from ..optim import HipAdam
    return {"sgd": torch.optim.SGD, "adam": HipAdam}


def rank_world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class Experiment(metaclass=ABCMeta):
    def __init__(self, config: dict, yamlConfig):
        self.base_config = BaseExperimentArgsModel(**config)
        if self.base_config.use_wandb:
            raise NotImplementedError("W&B logging needs network access; run with --use_wandb false")
        torch.manual_seed(self.base_config.seed)
        np.random.seed(self.base_config.seed)
        self.yaml_config = yamlConfig
        self.rank, self.world = rank_world()
        # the host torch seed stays equal on every rank (identical initial weights, identical host
        # LayerDrop draws in eager steps); the dropout masks and the device LayerDrop draws of captured
        # steps come from the functional seed stream, offset by the rank so that the ranks' halves of a
        # global batch draw independent masks, as one process would over its rows;
        # the device LayerDrop draws come from a stream without the offset (every rank skips alike)
        from .. import functional as Fn
        Fn.SEEDS.reseed(self.base_config.seed * 65537 + self.rank)
        Fn.LD_SEEDS.reseed(self.base_config.seed * 65537 + 7919)   # rank-independent (device LayerDrop)

        self.dataloader_train = self._create_dataloader(split="train")
        self.dataloader_val = self._create_dataloader(split="val")
        self.dataloader_test = self._create_dataloader(split="test")
        self.raw_config = config
        self.checkpoint_history = None

        stamp = f"{datetime.now():%Y-%m-%d_%H#%M#%S}"
        parts = [yamlConfig.cache_dir, "experiment_results", self.get_name()]
        if self.base_config.results_subdir_name is not None:
            parts.append(self.base_config.results_subdir_name)
        self.results_dir = os.path.join(*parts, stamp)
        if self.rank == 0:
            os.makedirs(self.results_dir, exist_ok=True)
            with open(os.path.join(self.results_dir, "config.json"), "w") as f:
                json.dump(dict(config, repro_cmd="python " + " ".join(sys.argv)), f, indent=5)

        from ..model.w2v_custom_feat_extractor import weights_loaded_later
        with weights_loaded_later(self.base_config.from_checkpoint is not None):
            self.model = self._create_model().cuda()
        if self.base_config.from_checkpoint is not None:
            print(f"loading model from checkpoint {self.base_config.from_checkpoint}")
            state = torch.load(self.base_config.from_checkpoint, map_location="cuda", weights_only=True)
            self.model.load_state_dict(state, strict=True)
            hist = os.path.join(os.path.dirname(self.base_config.from_checkpoint), "history.json")
            if os.path.exists(hist):
                print("Attempting to load history from checkpoint")
                try:
                    self.checkpoint_history = TrainHistory.from_json(hist)
                except (OSError, KeyError, ValueError, TypeError):
                    print("Failed to load history from checkpoint")

    # ------------------------------------------------------------------ run
    def run(self):
        from ..train.train_loop import Trainer
        trainer = Trainer(self)
        if not self.base_config.only_test:
            trained_model, history = trainer.train()
            if self.rank == 0:
                self.store_trained_model(trained_model)
                with open(os.path.join(self.results_dir, "history.json"), "w") as f:
                    json.dump(history.to_dict(), f, indent=5)
                self.plot_results(history)
                self.process_test_results(history.test_losses)
        else:
            test_results = self.run_real_world_test(self.model)
            if test_results is not None and self.rank == 0:
                self.process_test_results(test_results)
        print(f"Done. Saved results to {self.results_dir}")

    def store_trained_model(self, trained_model: torch.nn.Module):
        torch.save(trained_model.state_dict(), os.path.join(self.results_dir, "model.pt"))

    def process_test_results(self, test_results: SingleEpochHistory):
        pass

    def plot_results(self, history: TrainHistory):
        history.plot(os.path.join(self.results_dir, "history.png"))

    def run_real_world_test(self, model: B2TModel):
        res = self._predict_and_store(model, "test")
        if self.base_config.predict_on_train:
            self._predict_and_store(model, "train")
        return res

    # ------------------------------------------------------------------ hooks
    @abstractmethod
    def get_name(self) -> str:
        pass

    @abstractmethod
    def _create_dataset(self, split: Literal["train", "val", "test"] = "train"):
        raise NotImplementedError("Implement _create_dataset in subclass")

    @abstractmethod
    def _create_model(self) -> B2TModel:
        pass

    @staticmethod
    @abstractmethod
    def get_args_model() -> Type[BaseExperimentArgsModel]:
        raise NotImplementedError()

    @abstractmethod
    def get_vocab(self) -> list[str]:
        raise NotImplementedError("Implement get_vocab in subclass")

    @abstractmethod
    def create_evaluator(self, mode: Literal["train", "val", "test"], track_non_test_predictions: bool = False):
        raise NotImplementedError("Implement create_evaluator in subclass")

    def _create_dataloader(self, split: Literal["train", "val", "test"]) -> DataLoader:
        ds = self._create_dataset(split)
        sampler = self._dp_sampler(ds, split)
        return DataLoader(ds, batch_size=self.base_config.batch_size, shuffle=sampler is None,
                          sampler=sampler, collate_fn=ds.get_collate_fn())

    def _dp_sampler(self, ds, split):
        """Data-parallel runs shard the train split across ranks (each rank a disjoint 1/world)."""
        if self.world > 1 and split == "train":
            from torch.utils.data.distributed import DistributedSampler
            return DistributedSampler(ds, num_replicas=self.world, rank=self.rank, shuffle=True,
                                      seed=self.base_config.seed, drop_last=True)
        return None

    def _get_optimizer_cls(self) -> type:
        opts = _optimizers()
        if self.base_config.optimizer not in opts:
            raise ValueError(f"Optimizer {self.base_config.optimizer} not implemented. Choose from {list(opts)} "
                             "or implement your own.")
        return opts[self.base_config.optimizer]

    def create_optimizer(self) -> Optimizer:
        cls: Any = self._get_optimizer_cls()
        return cls(self.model.parameters(), lr=self.base_config.learning_rate,
                   weight_decay=self.base_config.weight_decay, eps=self.base_config.optimizer_epsilon)

    def get_scheduler(self, optimizer: Optimizer):
        return torch.optim.lr_scheduler.StepLR(optimizer, step_size=self.base_config.scheduler_step_size,
                                               gamma=self.base_config.scheduler_gamma)

    # ------------------------------------------------------------------ prediction
    def _predict_and_store(self, model: B2TModel, mode: Literal["train", "test"]):
        def on_batch(batch_id: int, batch: SampleBatch, outputs: ModelOutput):
            if batch_id >= self.base_config.visualize_predictions_n_batches:
                return
            out_dir = os.path.join(self.results_dir, f"{mode}_predictions")
            os.makedirs(out_dir, exist_ok=True)
            self.visualize_predictions(batch, outputs, os.path.join(out_dir, f"batch_{batch_id}.png"), batch_id)

        pred = self._predict(model, mode, on_batch)
        if pred is not None and self.rank == 0:
            with open(os.path.join(self.results_dir, f"{mode}_predictions.json"), "w") as f:
                json.dump(pred.to_dict(), f, indent=5)
        return pred

    def _predict(self, model: B2TModel, mode: Literal["train", "test"],
                 handle_prediction_batch: Optional[Callable[[int, SampleBatch, ModelOutput], Any]] = None):
        loader = self.dataloader_train if mode == "train" else self.dataloader_test
        evaluator = self.create_evaluator(mode, True)
        model.eval()
        for i, data in enumerate(loader):
            data = cast(SampleBatch, data).cuda()
            with torch.no_grad():
                outputs = model.forward(data)
                if outputs.logits.shape[0] == 0:
                    print("Skipping _predict because outputs don't have logits")
                    return None
                evaluator.track_batch(outputs, data)
                if handle_prediction_batch is not None:
                    handle_prediction_batch(i, data, outputs)
        result = evaluator.evaluate()
        evaluator.clean_up()
        return result

    def visualize_predictions(self, batch: SampleBatch, output: ModelOutput, out_path: str, batch_id: int):
        """Per-frame class probabilities of up to 4 samples as a table heat map (reference :265-346)."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        from matplotlib.colors import Normalize
        vocab = self.get_vocab()
        probs = output.logits.softmax(-1).cpu().numpy()
        pred = ["".join(vocab[i] for i in np.argmax(p, axis=-1)) for p in probs]
        tgt = ["".join(vocab[i] for i in t) for t in batch.target.tolist()] if batch.target is not None else None
        bsz, T, V = probs.shape
        px = 1 / plt.rcParams["figure.dpi"]
        rows = min(bsz, 4)
        fig, axs = plt.subplots(nrows=rows, figsize=(T * 18 * px, (V + 1) * 1.5 * rows * 18 * px))
        axs = axs if rows > 1 else [axs]
        norm = Normalize(vmin=0, vmax=1)
        for s, ax in enumerate(axs):
            table = ax.table(cellText=[[vocab[r]] * T for r in range(V)], cellLoc="center", loc="center",
                             cellColours=plt.cm.Blues(norm(probs[s].T)))
            for t in range(T):
                cell = table[int(np.argmax(probs[s][t])), t]
                cell.set_edgecolor("red")
                cell.set_linewidth(2)
            table.auto_set_font_size(False)
            table.set_fontsize(8)
            ax.set_xticks([])
            ax.set_yticks([])
            ax.set_xlabel(f"Target: {tgt[s] if tgt is not None else None}\nPrediction: {pred[s]}")
        plt.title(f"Displaying {rows}/{bsz} samples")
        plt.tight_layout()
        plt.savefig(out_path)
        plt.close(fig)
