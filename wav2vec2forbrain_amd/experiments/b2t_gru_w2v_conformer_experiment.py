"""b2p2t_gru+w2v_conformer — mirrors reference src/experiments/b2t_gru_w2v_conformer_experiment.py:36-178:
the B2P2T GRU brain encoder feeding the wav2vec2-conformer (rotary) encoder + CTC head; optimizer,
schedules and evaluator as in the w2v experiment (the reference duplicates them)."""
from __future__ import annotations

from typing import Any, Literal, Optional, cast

from pydantic import Field
from torch.optim.optimizer import Optimizer

from ..model.brain_feature_extractor import B2P2TBrainFeatureExtractorArgsModel, bfe_w_preprocessing_from_config
from ..model.w2v_conformer_custom_feat_extractor import W2VConformerBrainEncoderModel
from ..train.evaluator import EvaluatorWithW2vLMDecoder
from .b2t_experiment import B2TArgsModel, B2TExperiment
from .b2t_gru_w2v_experiment import (DEFAULT_BEAM_WIDTH, DEFAULT_MIN_TOKEN_LOGP, DEFAULT_PRUNE_LOGP,
                                     trainable_param_groups, w2v_scheduler)

W2V_CHECKPOINT_TO_PROCESSOR = {
    "facebook/wav2vec2-conformer-rope-large-960h-ft": "patrickvonplaten/wav2vec2-base-100h-with-lm",
}


class B2TGruAndW2VConformerArgsModel(B2TArgsModel, B2P2TBrainFeatureExtractorArgsModel):
    brain_encoder_path: Optional[str] = None
    unfreeze_strategy: Literal["brain_encoder", "brain_encoder+w2v"] = "brain_encoder"
    w2v_learning_rate: Optional[float] = None
    w2v_warmup_start_step: Optional[int] = Field(default=None, description=(
        "Epoch at which warm up phase of w2v lr starts. Before LR will be 0. 0 if not provided"))
    w2v_warmup_steps: Optional[int] = Field(default=None, description=(
        "Num epochs from w2v_warmup_start_step to reach full w2v_learning_rate. 0 if not provided"))
    wav2vec_checkpoint: str = "facebook/wav2vec2-conformer-rope-large-960h-ft"
    lm_decode_test_predictions: bool = False
    adjust_global_lr_to_w2v_postwarmup_lr: Optional[bool] = Field(default=None, description=(
        "Adjust the global learning rate to that of w2v over w2v warmup interval, then keep at w2v_learning_rate. "
        "Only valid when brain_encoder+w2v unfreeze strategy is set."))
    lm_decode_beam_width: int = DEFAULT_BEAM_WIDTH
    lm_decode_beam_prune_logp: float = DEFAULT_PRUNE_LOGP
    lm_decode_token_min_logp: float = DEFAULT_MIN_TOKEN_LOGP
    lm_decode_alpha: float = 0.5
    lm_decode_beta: float = 0.5
    lm_score_boundary: bool = False
    # build addition: synchronised BatchNorm statistics across data-parallel ranks
    sync_batchnorm: bool = True


class B2TGruAndW2VConformerExperiment(B2TExperiment):
    def __init__(self, config: dict, yamlConfig):
        self.config = self.get_args_model()(**config)
        super().__init__(config, yamlConfig)
        if self.config.tokenizer_checkpoint != self.config.wav2vec_checkpoint:
            print(f"Tokenizer checkpoint ({self.config.tokenizer_checkpoint}) is different to wav2vec_checkpoint "
                  f"({self.config.wav2vec_checkpoint}). This may lead to unexpected behaviour")

    def get_name(self) -> str:
        return "b2p2t_gru+w2v_conformer"

    @staticmethod
    def get_args_model():
        return B2TGruAndW2VConformerArgsModel

    def _create_model(self):
        brain_encoder = bfe_w_preprocessing_from_config(self.config, self.config.brain_encoder_path,
                                                        self.config.wav2vec_checkpoint)
        model = W2VConformerBrainEncoderModel(brain_encoder, self.config.wav2vec_checkpoint)
        model.sync_batchnorm = self.config.sync_batchnorm
        return model

    def create_optimizer(self) -> Optimizer:
        cls: Any = self._get_optimizer_cls()
        return cls(trainable_param_groups(cast(W2VConformerBrainEncoderModel, self.model), self.config),
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
