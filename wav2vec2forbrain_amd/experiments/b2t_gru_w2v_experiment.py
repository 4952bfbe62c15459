"""b2p2t_gru+w2v — mirrors reference src/experiments/b2t_gru_w2v_experiment.py:41-207: the B2P2T
GRU brain encoder feeding the wav2vec2 encoder + CTC head, Adam over the brain encoder (or over
brain encoder + w2v with its own learning rate), StepLR or the two-module warmup schedule, the
greedy-decode evaluator with CER, model.pt + brain_encoder.pt artefacts."""
from __future__ import annotations

import os
from typing import Any, Literal, Optional, cast

import torch
from pydantic import Field
from torch.optim.optimizer import Optimizer

from ..model.brain_feature_extractor import B2P2TBrainFeatureExtractorArgsModel, bfe_w_preprocessing_from_config
from ..model.w2v_custom_feat_extractor import W2VBrainEncoderModel, W2VBrainEncoderModelArgs
from ..train.evaluator import EvaluatorWithW2vLMDecoder
from ..util.warmup_scheduler import get_2module_warmup_scheduler
from .b2t_experiment import B2TArgsModel, B2TExperiment

# pyctcdecode.constants defaults (DEFAULT_BEAM_WIDTH, DEFAULT_PRUNE_LOGP, DEFAULT_MIN_TOKEN_LOGP)
DEFAULT_BEAM_WIDTH = 100
DEFAULT_PRUNE_LOGP = -10.0
DEFAULT_MIN_TOKEN_LOGP = -5.0

W2V_CHECKPOINT_TO_PROCESSOR = {
    "facebook/wav2vec2-base-960h": "patrickvonplaten/wav2vec2-base-100h-with-lm",
    "facebook/wav2vec2-base-100h": "patrickvonplaten/wav2vec2-base-100h-with-lm",
    "jonatasgrosman/wav2vec2-large-xlsr-53-english": "jonatasgrosman/wav2vec2-large-xlsr-53-english",
    "facebook/wav2vec2-large-960h": "patrickvonplaten/wav2vec2-base-100h-with-lm",
}


class B2TGruAndW2VArgsModel(B2TArgsModel, B2P2TBrainFeatureExtractorArgsModel, W2VBrainEncoderModelArgs):
    brain_encoder_path: Optional[str] = None
    unfreeze_strategy: Literal["brain_encoder", "brain_encoder+w2v"] = "brain_encoder"
    w2v_learning_rate: Optional[float] = None
    w2v_warmup_start_step: Optional[int] = Field(default=None, description=(
        "Epoch at which warm up phase of w2v lr starts. Before LR will be 0. 0 if not provided"))
    w2v_warmup_steps: Optional[int] = Field(default=None, description=(
        "Num epochs from w2v_warmup_start_step to reach full w2v_learning_rate. 0 if not provided"))
    wav2vec_checkpoint: str = "facebook/wav2vec2-base-960h"
    lm_decode_test_predictions: bool = False
    adjust_global_lr_to_w2v_postwarmup_lr: Optional[bool] = Field(default=None, description=(
        "Adjust the global learning rate to that of w2v over w2v warmup interval, then keep at w2v_learning_rate. "
        "Only valid when brain_encoder+w2v unfreeze strategy is set."))
    w2v_skip_loading_weights: bool = Field(default=False, description=(
        "Skip loading weights from wav2vec checkpoint, only load architecture"))
    lm_decode_beam_width: int = DEFAULT_BEAM_WIDTH
    lm_decode_beam_prune_logp: float = DEFAULT_PRUNE_LOGP
    lm_decode_token_min_logp: float = DEFAULT_MIN_TOKEN_LOGP
    lm_decode_alpha: float = 0.5
    lm_decode_beta: float = 0.5
    lm_score_boundary: bool = False
    store_brain_encoder: bool = Field(default=False, description=(
        "Store brain encoder model seperate from whole model in results directory"))


def trainable_param_groups(model, config):
    """brain_encoder only, or brain_encoder + w2v_encoder (lr = w2v_learning_rate or learning_rate)."""
    if config.unfreeze_strategy == "brain_encoder+w2v":
        return [{"params": model.brain_encoder.parameters()},
                {"params": model.w2v_encoder.parameters(),
                 "lr": config.w2v_learning_rate if config.w2v_learning_rate is not None else config.learning_rate}]
    if config.unfreeze_strategy == "brain_encoder":
        assert config.w2v_learning_rate is None, \
            "w2v_learning_rate can only be set if unfreeze strategy is brain_encoder+w2v"
        return model.brain_encoder.parameters()
    raise Exception(f"Unfreeze strategy {config.unfreeze_strategy} is not implemented for wav2vec experiment")


def w2v_scheduler(experiment, optimizer):
    """StepLR (brain_encoder) or the two-module LambdaLR warmup (brain_encoder+w2v)."""
    c = experiment.config
    if c.unfreeze_strategy == "brain_encoder":
        assert c.w2v_warmup_steps is None, "w2v_warmup_steps can only be set if unfreeze strategy is brain_encoder+w2v"
        assert c.adjust_global_lr_to_w2v_postwarmup_lr is None, \
            "adjust_global_lr_to_w2v_postwarmup_lr can only be set if unfreeze strategy is brain_encoder+w2v"
        return torch.optim.lr_scheduler.StepLR(optimizer, step_size=experiment.base_config.scheduler_step_size,
                                               gamma=experiment.base_config.scheduler_gamma)
    return get_2module_warmup_scheduler(
        optimizer, c.learning_rate, c.w2v_warmup_start_step or 0, c.w2v_warmup_steps or 0,
        c.w2v_learning_rate if c.w2v_learning_rate is not None else c.learning_rate,
        c.adjust_global_lr_to_w2v_postwarmup_lr is True)


class B2TGruAndW2VExperiment(B2TExperiment):
    def __init__(self, config: dict, yamlConfig):
        self.config = self.get_args_model()(**config)
        super().__init__(config, yamlConfig)
        if self.config.tokenizer_checkpoint != self.config.wav2vec_checkpoint:
            print(f"Tokenizer checkpoint ({self.config.tokenizer_checkpoint}) is different to wav2vec_checkpoint "
                  f"({self.config.wav2vec_checkpoint}). This may lead to unexpected behaviour")

    def get_name(self) -> str:
        return "b2p2t_gru+w2v"

    @staticmethod
    def get_args_model():
        return B2TGruAndW2VArgsModel

    def _create_model(self):
        brain_encoder = bfe_w_preprocessing_from_config(self.config, self.config.brain_encoder_path,
                                                        self.config.wav2vec_checkpoint)
        return W2VBrainEncoderModel(self.config, brain_encoder, self.config.wav2vec_checkpoint, None,
                                    self.config.w2v_skip_loading_weights)

    def create_optimizer(self) -> Optimizer:
        cls: Any = self._get_optimizer_cls()
        return cls(trainable_param_groups(cast(W2VBrainEncoderModel, self.model), self.config),
                   lr=self.base_config.learning_rate, weight_decay=self.base_config.weight_decay,
                   eps=self.base_config.optimizer_epsilon)

    def get_scheduler(self, optimizer: Optimizer):
        return w2v_scheduler(self, optimizer)

    def create_evaluator(self, mode: Literal["train", "val", "test"], track_non_test_predictions: bool = False):
        c = self.config
        return EvaluatorWithW2vLMDecoder(
            self.tokenizer, mode, self.yaml_config.cache_dir, W2V_CHECKPOINT_TO_PROCESSOR.get(c.wav2vec_checkpoint, ""),
            track_non_test_predictions, c.lm_decode_test_predictions, c.lm_decode_beam_width,
            c.lm_decode_beam_prune_logp, c.lm_decode_token_min_logp, c.lm_decode_alpha, c.lm_decode_beta,
            c.lm_score_boundary)

    def store_trained_model(self, trained_model: W2VBrainEncoderModel):
        super().store_trained_model(trained_model)
        torch.save(trained_model.brain_encoder.state_dict(), os.path.join(self.results_dir, "brain_encoder.pt"))
