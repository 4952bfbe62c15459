"""Trainer — mirrors reference src/train/train_loop.py:14-220 (the per-batch body :41-84 is the
hot path; W&B logging is not available offline and is omitted). Data-parallel when
torch.distributed is initialised: gradients of the optimised parameters are all-reduced by
train.ddp.GradBucketReducer overlapped with backward."""
from __future__ import annotations

import contextlib
import dataclasses
import os
import sys
import uuid
from typing import Literal, cast

import numpy as np
import torch

from .. import functional as Fn
import torch.distributed as dist

from ..datasets.batch_types import SampleBatch
from .ddp import GradBucketReducer, collectives_in_graph, dp_active, unused_param_names
from .history import EpochLosses, SingleEpochHistory, TrainHistory


def _detached(out):
    """The step's ModelOutput with its tensors detached. After backward the caller only reads values
    (evaluator: loss, logits); a returned output that still referenced the autograd graph would keep
    the parameters' AccumulateGrad nodes alive, bound to the stream they were created on, and the next
    step's capture on the capture stream would then accumulate through them (an illegal cross-stream
    dependency inside the capture: the HIP runtime crashed in hipStreamEndCapture)."""
    return dataclasses.replace(out, **{f.name: getattr(out, f.name).detach() for f in dataclasses.fields(out)
                                       if isinstance(getattr(out, f.name), torch.Tensor)})


class Trainer:
    def __init__(self, experiment):
        self.experiment = experiment
        self.config = experiment.base_config
        self.dataloader_train = experiment.dataloader_train
        self.dataloader_val = experiment.dataloader_val
        self.dataloader_test = experiment.dataloader_test
        self.model = experiment.model
        self.optimizer = experiment.create_optimizer()
        self.scheduler = experiment.get_scheduler(self.optimizer)
        self.reducer = None
        self.frozen_reducer = None
        opt_ids = {id(p) for g in self.optimizer.param_groups for p in g["params"]}
        # frozen parameters (not optimised): their gradient GEMMs run deferred beside the GRU backward
        Fn.set_deferred_wgrad(self._setup_dp(opt_ids), names=self._param_names())
        # precision policy of the default (bf16) mode: with the w2v encoder trained (full fine-tuning,
        # unfreeze_strategy=brain_encoder+w2v) the step runs in the bf16x3 mode. Adam's first updates of
        # the ~600 M encoder parameters are ~lr * sign(g), and the 16-bit operands' rounding (bf16 or fp16,
        # forward or backward) moved the 3-step CTC-loss trajectory 1.3e-3 .. 7.4e-3 away from the
        # reference's; split-bf16 GEMMs hold it at 1.3e-4 (tools/traj_err_ft.py).
        # B2P_TRAIN_PRECISION: auto (this policy) | keep (the ambient mode as it is)
        enc = getattr(self.model, "w2v_encoder", None)
        self.encoder_trained = enc is not None and any(id(p) in opt_ids for p in enc.parameters())
        self.precision_policy = os.environ.get("B2P_TRAIN_PRECISION", "auto")
        # replayed steps (see train_step): a cache of captured steps keyed by the batch shape
        self.use_graphs = (os.environ.get("B2P_TRAINER_GRAPH", "1") != "0" and torch.cuda.is_available()
                           and hasattr(self.optimizer, "make_capturable"))
        self.graph_cache_size = int(os.environ.get("B2P_TRAINER_GRAPHS", "4"))
        self.capture_after = int(os.environ.get("B2P_TRAINER_CAPTURE_AFTER", "1"))
        # data-parallel replays capture the step in segments split at its collectives (SyncBN
        # statistics, gradient buckets); 0: one graph, SyncBN steps eager, buckets after the replay
        self.segmented = os.environ.get("B2P_SEGMENTED_CAPTURE", "1") != "0"
        self._graphs: dict = {}
        self._opt_generation = getattr(self.optimizer, "generation", 0)
        self._shape_seen: dict = {}
        self._capture_failed: dict = {}   # batch shape -> the capture error (data-parallel fallback)
        self._epoch_counter = None
        self.graph_steps = 0
        self.eager_steps = 0

    def _param_names(self) -> dict:
        return {id(p): n for n, p in self.model.named_parameters()}

    def _setup_dp(self, opt_ids: set) -> list:
        """(Re)builds the data-parallel machinery for the optimised parameter set opt_ids: the bucket
        reducer of the optimised gradients, the frozen-gradient reducer and the optimizer's device gates.
        Returns the frozen (trainable, not optimised) parameters. Called again when the optimizer gains a
        param group (HipAdam.add_param_group), so the new group's gradients are all-reduced and gated
        like the others."""
        for r in (self.reducer, self.frozen_reducer):
            if r is not None:
                r.close()
        self.reducer = self.frozen_reducer = None
        frozen = [p for p in self.model.parameters() if p.requires_grad and id(p) not in opt_ids]
        if dp_active():
            skip = unused_param_names(self.model)
            params = [p for n, p in self.model.named_parameters() if id(p) in opt_ids and n not in skip]
            self.reducer = GradBucketReducer(params, bucket_mb=float(os.environ.get("B2P_DP_BUCKET_MB", "64")))
            if hasattr(self.optimizer, "make_capturable"):
                # device-form update gated per parameter by "some rank used it" (LayerDrop: a
                # parameter no rank used keeps its value and moments, as with grad=None)
                self.optimizer.make_capturable(params[0].device)
                self.optimizer.gates = self.reducer.gates
            if self.config.gradient_clipping is not None:
                # clip_grad_norm_ runs over model.parameters() (reference :72-75), frozen gradients
                # included; averaging those too keeps every rank's clip coefficient equal to the
                # single-process global-batch one (they accumulate across steps identically on all
                # ranks once averaged, so averaging the running sum each step is exact)
                self.frozen_reducer = GradBucketReducer(frozen, overlap=False, grad_views=False, track_used=False)
        return frozen

    def _log_intermediate(self, batch: int, n_batches: int, evaluator):
        print(f"Batch {batch + 1}/{n_batches} loss: {evaluator.get_latest_loss():.2f} "
              f"running: {evaluator.get_running_loss():.2f}\r", end="")

    # ------------------------------------------------------------------ replayed steps
    @staticmethod
    def _shape_key(batch):
        t = batch.target
        return (tuple(batch.input.shape), None if t is None else tuple(t.shape), str(batch.input.device))

    def _sync_bn(self) -> bool:
        """Data-parallel with synchronised BatchNorm statistics (the Conformer's sync_batchnorm): the
        statistics all-reduces run inside the forward and backward. A captured step cannot hold a
        collective, so the data-parallel step is captured in segments split at each of them
        (train/step_graph.py); B2P_SEGMENTED_CAPTURE=0 keeps such steps eager instead. With
        sync_batchnorm off each rank normalises over its own micro-batch (torch DDP's default
        semantics) in eager and replayed steps alike."""
        return self.reducer is not None and any(getattr(m, "sync_batchnorm", False) for m in self.model.modules())

    def _graphable(self, batch) -> bool:
        return (self.use_graphs and self.model.training and batch.input.is_cuda and batch.target is not None
                and getattr(batch, "target_lens", None) is not None and not Fn.capturing()
                and (self.segmented or not self._sync_bn() or collectives_in_graph()))

    def _capture(self, batch):
        """Captures one whole step for this batch shape (train/step_graph.py) on static copies of the
        batch tensors; the captured step reads them, train_step copies each new batch into them."""
        from .step_graph import StepGraph
        static = batch.copy_and_change(**{f: getattr(batch, f).clone() for f in batch._fields
                                          if isinstance(getattr(batch, f), torch.Tensor)})
        for a in ("day_idxs", "input_lens", "target_lens"):
            v = getattr(batch, a, None)
            if isinstance(v, torch.Tensor):
                setattr(static, a, v.clone())
        mods = [m for m in self.model.modules() if hasattr(m, "sync_metrics")]
        olds = [m.sync_metrics for m in mods]
        for m in mods:   # no host sync inside the captured step: the loss stays a device tensor
            m.sync_metrics = False
        box = {}
        dp = self.reducer is not None
        # RCCL: the whole data-parallel step is ONE graph: the step's collectives (SyncBN statistics, the
        # gradient buckets as they complete during the backward, the used-flag MAX) are captured inside
        # it, and so are the clip and the Adam update. gloo: segmented capture (a gloo collective is host
        # code): the graph splits at every collective, which a replay issues between the segments
        in_graph = dp and collectives_in_graph()
        seg = dp and self.segmented and not in_graph

        def step():
            out = self._eager_body(static, in_graph=True)
            if in_graph:
                # the exchange tail inside the capture: remaining buckets, the used flags of this replay's
                # LayerDrop draw (device flags), waits (stream joins), clip, update
                self.reducer.use_layer_gates(self.reducer.make_layer_gates(Fn.layerdrop_param_gates()))
                try:
                    self.reducer.finish()
                finally:
                    self.reducer.use_layer_gates(None)
                if self.frozen_reducer is not None:
                    self.frozen_reducer.finish()
                if self.config.gradient_clipping is not None:
                    torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.config.gradient_clipping)
                self.optimizer.step()   # the device form (StepGraph made it capturable)
            box["out"] = out
            return out.loss.detach().reshape(1)

        if self._epoch_counter is None:
            self._epoch_counter = torch.zeros(1, dtype=torch.int64, device=batch.input.device)
        if dp:
            # bucket all-reduces from the backward hooks: inside the one RCCL graph they run on RCCL's
            # stream beside the rest of the backward (the frozen-weight side streams are joined before the
            # tail, so nothing waits for them early); segmented (gloo) only when no frozen-weight gradient
            # work runs on the side streams (full fine-tuning): a split joins those streams, which would
            # serialise them with the GRU backward they are meant to run beside. Otherwise every bucket is
            # exchanged after the replay (finish()).
            self.reducer.overlap = in_graph or (seg and not Fn.deferred_wgrad_active())
        try:
            sg = StepGraph(step, None if (dp and not in_graph) else self.optimizer, warmup=0, warm_replays=0,
                           epoch=self._epoch_counter, segmented=seg)
            sg.capture()
        finally:
            if dp:
                self.reducer.overlap = True
                self.reducer._reset()
            for m, o in zip(mods, olds):
                m.sync_metrics = o
        gates = self.reducer.make_layer_gates(Fn.layerdrop_param_gates()) if (dp and not in_graph) else None
        return dict(graph=sg, batch=static, out=box["out"], gates=gates, sync=any(olds), tail=dp and not in_graph)

    def _replay(self, g, batch):
        st = g["batch"]
        for f in batch._fields:
            v = getattr(batch, f)
            if isinstance(v, torch.Tensor):
                getattr(st, f).copy_(v, non_blocking=True)
        for a in ("day_idxs", "input_lens", "target_lens"):
            v = getattr(batch, a, None)
            if isinstance(v, torch.Tensor):
                getattr(st, a).copy_(v, non_blocking=True)
        g["graph"].replay()
        if g["tail"]:   # gloo: exchange, clip and update after the replay
            self.reducer.use_layer_gates(g["gates"])
            self._dp_tail()
        # the captured output's tensors are overwritten by the next replay
        out = dataclasses.replace(g["out"], metrics=dict(g["out"].metrics))
        if g["sync"] and "ctc_loss" in out.metrics:
            # the reference reads ctc_loss.item() every step (w2v_custom_feat_extractor.py:94); the
            # same transfer carries the multi-CU GRU status word (raises on a recurrence timeout)
            out.metrics["ctc_loss"] = Fn.loss_item(out.loss)
        return out

    def _dp_tail(self):
        """After a replayed forward + backward: bucket exchange, clip, update (eager)."""
        self.reducer.finish()
        if self.frozen_reducer is not None:
            self.frozen_reducer.finish()
        if self.config.gradient_clipping is not None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.config.gradient_clipping)
        self.optimizer.step()
        self.reducer.use_layer_gates(None)

    def release_graphs(self) -> None:
        for g in self._graphs.values():
            g["graph"].release()
        self._graphs.clear()

    def step_precision(self) -> str | None:
        """The precision mode this Trainer's steps run in under the policy (None: the ambient mode)."""
        if self.precision_policy == "auto" and self.encoder_trained and Fn.bf16_mode():
            return "bf16x3"
        return None

    def train_step(self, batch: SampleBatch):
        gen = getattr(self.optimizer, "generation", 0)
        if gen != self._opt_generation:
            # the optimizer gained a param group (HipAdam.add_param_group): steps captured before hold
            # update records for the old groups only, so they are dropped and captured again
            self.release_graphs()
            self._opt_generation = gen
            opt_ids = {id(p) for g in self.optimizer.param_groups for p in g["params"]}
            # data-parallel: the new group's gradients join the bucket reducer (and leave the frozen one),
            # and the optimizer's gates follow the new parameter list
            Fn.set_deferred_wgrad(self._setup_dp(opt_ids), names=self._param_names())
            enc = getattr(self.model, "w2v_encoder", None)
            self.encoder_trained = enc is not None and any(id(p) in opt_ids for p in enc.parameters())
        with self.precision_context():
            return self._train_step(batch)

    def precision_context(self):
        """The precision mode of this Trainer's steps (step_precision) and, in the bf16x3 policy, its
        per-role GEMM forms (functional.X3_POLICY_FORMS)."""
        mode = self.step_precision()
        stack = contextlib.ExitStack()
        if mode is not None:
            stack.enter_context(Fn.precision(mode))
            if mode == "bf16x3":
                stack.enter_context(Fn.x3_forms(Fn.X3_POLICY_FORMS))
        return stack

    def _train_step(self, batch: SampleBatch):
        """One training step. The first `capture_after` steps of a batch shape run eagerly; then the
        whole step is captured once as a HIP graph and replayed for every later batch of that shape
        (at most graph_cache_size shapes; other shapes keep running eagerly). Replayed and eager steps
        compute the same update (tests/test_trainer_gpu.py); the replay issues it with one host call
        instead of ~650 Python-issued launches."""
        if self._graphable(batch):
            key = self._shape_key(batch)
            g = self._graphs.get(key)
            if g is None:
                n = self._shape_seen.get(key, 0)
                self._shape_seen[key] = n + 1
                if (n >= self.capture_after and len(self._graphs) < self.graph_cache_size
                        and key not in self._capture_failed):
                    try:
                        g = self._graphs[key] = self._capture(batch)
                    except Exception as e:   # noqa: BLE001
                        # a data-parallel capture that fails (the in-graph RCCL form has run at world size 1
                        # only, on the boxes this was built on) leaves this batch shape on eager steps, which
                        # compute the same update, instead of ending the run; B2P_CAPTURE_FALLBACK=0 raises
                        if self.reducer is None or os.environ.get("B2P_CAPTURE_FALLBACK", "1") == "0":
                            raise
                        self._capture_failed[key] = repr(e)
                        print(f"Trainer: step capture failed for batch shape {key[0]} ({e!r}); eager steps",
                              file=sys.stderr, flush=True)
                        g = None
            if g is not None:
                self.graph_steps += 1
                return self._replay(g, batch)
        self.eager_steps += 1
        if self.reducer is not None:
            self.reducer.use_layer_gates(None)
        return self._eager_body(batch)

    def _eager_body(self, batch: SampleBatch, in_graph: bool = False):
        """One step of the reference loop body (:42-79): zero_grad, (no-op noise), forward,
        backward, [DP all-reduce], optional clip, optimizer step. in_graph (captured data-parallel
        step): stops after the backward; the exchange and update run after each replay."""
        if self.reducer is not None:
            self.reducer.zero_grad()    # trainable gradients live in the all-reduce buckets
        else:
            self.optimizer.zero_grad()
        if self.config.whiteNoiseSD > 0:       # reference :46-52: computed and discarded
            _ = torch.randn(batch.input.shape, device=batch.input.device) * self.config.whiteNoiseSD
        if self.config.constantOffsetSD > 0:   # reference :54-62: computed and discarded
            inp = batch.input
            _ = torch.randn([inp.shape[0], 1, inp.shape[2]], device=inp.device) * self.config.constantOffsetSD
        with torch.enable_grad():
            outputs = self.model.forward(batch)
        loss = cast(torch.Tensor, outputs.loss)
        loss.backward(Fn.loss_seed(loss))   # = loss.backward(): the seed is a cached ones tensor
        Fn.join_wgrad()
        if in_graph and self.reducer is not None:
            return _detached(outputs)
        if self.reducer is not None:
            self.reducer.finish()
        if self.frozen_reducer is not None:
            self.frozen_reducer.finish()
        if self.config.gradient_clipping is not None:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.config.gradient_clipping)
        self.optimizer.step()
        return _detached(outputs)

    def _train_epoch(self, data_loader, epoch: int = 0):
        self.model.train()
        sampler = getattr(data_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            # DistributedSampler: a new permutation (and per-rank shard) every epoch, as the
            # reference's single-process DataLoader(shuffle=True) reshuffles every epoch
            sampler.set_epoch(epoch)
        evaluator = self.experiment.create_evaluator("train")
        for i, batch in enumerate(data_loader):
            batch = cast(SampleBatch, batch).cuda()
            outputs = self.train_step(batch)
            evaluator.track_batch(outputs, batch)
            if i % self.config.log_every_n_batches == self.config.log_every_n_batches - 1:
                self._log_intermediate(i, len(data_loader), evaluator)
        results = evaluator.evaluate()
        evaluator.clean_up()
        return results

    def _evaluate_epoch(self, mode: Literal["val", "test"]):
        dataloader = self.dataloader_val if mode == "val" else self.dataloader_test
        self.model.eval()
        evaluator = self.experiment.create_evaluator(mode)
        for i, batch in enumerate(dataloader):
            batch = cast(SampleBatch, batch).cuda()
            with torch.no_grad():
                outputs = self.model.forward(batch)
            evaluator.track_batch(outputs, batch)
        results = evaluator.evaluate()
        evaluator.clean_up()
        return results

    def train(self):
        history: list[EpochLosses] = (list(self.experiment.checkpoint_history.epochs)
                                      if self.experiment.checkpoint_history is not None else [])
        best = float("inf" if self.config.minimize_best_model_metric else "-inf")
        best_path = os.path.join(self.experiment.yaml_config.cache_dir, "model_checkpoints", str(uuid.uuid4()),
                                 "best_model.pt")
        os.makedirs(os.path.dirname(best_path), exist_ok=True)

        def metric(h: SingleEpochHistory):
            avg = h.get_average()
            return avg.loss if self.config.best_model_metric == "loss" else avg.metrics[self.config.best_model_metric]

        saved = False
        for epoch in range(self.config.epochs):
            print(f"\nEpoch {epoch + 1}/{self.config.epochs}")
            train_losses = self._train_epoch(self.dataloader_train, epoch)
            val_losses = self._evaluate_epoch("val")
            self.scheduler.step()
            print(f"\n\n{'=' * 20}\nFinished Epoch {epoch + 1}/{self.config.epochs} "
                  f"train {self.config.loss_function}-loss: {train_losses.get_average().loss} "
                  f"val {self.config.loss_function}-loss: {val_losses.get_average().loss}")
            history.append(EpochLosses(train_losses, val_losses))
            if self.config.return_best_model:
                cur = metric(val_losses)
                if (cur < best) if self.config.minimize_best_model_metric else (cur > best):
                    best = cur
                    torch.save(self.model.state_dict(), best_path)
                    saved = True
                    print(f"\n\nSaving model checkpoint at {best_path}\n")
            patience = self.config.early_stopping_patience
            if patience is not None and len(history) >= patience:
                recent = [metric(e.val_losses) for e in history][-patience:]
                # the oldest of the window, shifted by the delta, is the baseline to beat
                recent[0] += -self.config.early_stopping_delta if self.config.minimize_best_model_metric \
                    else self.config.early_stopping_delta
                bi = np.argmin(recent) if self.config.minimize_best_model_metric else np.argmax(recent)
                if bi == 0:
                    print(f"\nEarly stopping after {epoch} epochs ({patience} epochs without improvement in "
                          f"validation {self.config.best_model_metric} metrics)")
                    break
        if self.config.return_best_model and saved:
            self.model.load_state_dict(torch.load(best_path, weights_only=True))
            os.remove(best_path)
            os.rmdir(os.path.dirname(best_path))
            print("Loaded model with best validation loss of this experiment from disk")
        if getattr(self.config, "train_on_val_once", False):   # reference :211-213
            print("Training one epoch on val set")
            self._train_epoch(self.dataloader_val, self.config.epochs)
        test_losses = self._evaluate_epoch("test")
        print(f"\nTest loss ({self.config.loss_function}): {test_losses.get_average().loss}")
        return self.model, TrainHistory(history, test_losses)
