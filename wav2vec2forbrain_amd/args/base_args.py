"""Argument models shared by the experiments — mirrors reference src/args/base_args.py:5-134
(pydantic models; the reference uses pydantic v1, this build runs on v2 with the same fields)."""
from __future__ import annotations

from typing import Literal, Optional

from pydantic import BaseModel, Field

PRETRAINED_LATENT_SIZES = {
    "jonatasgrosman/wav2vec2-large-xlsr-53-english": 1024,
    "facebook/wav2vec2-base-960h": 768,
    "facebook/wav2vec2-large-960h": 1024,
    "facebook/wav2vec2-conformer-rope-large-960h-ft": 1024,
    "facebook/wav2vec2-lv-60-espeak-cv-ft": 1024,
}


class B2TDatasetArgsModel(BaseModel):
    preprocessing: Literal[
        "competition_recommended", "seperate_zscoring", "only_tx_unnormalized", "only_tx_zscored",
        "only_spikepow_unnormalized", "only_spikepow_zscored", "seperate_zscoring_2channels",
        "seperate_zscoring_4channels",
    ] = "seperate_zscoring"
    competition_mode: bool = False
    limit_samples: Optional[int] = Field(default=None, description="Limit number of samples")
    sample_rate: int = 50
    remove_punctuation: bool = True
    area: Literal["6v", "44"] = "6v"


class BaseExperimentArgsModel(BaseModel):
    batch_size: int = Field(16, description="Batch size for training and validation")
    epochs: int = 10
    learning_rate: float = 0.001
    optimizer: Literal["adam", "sgd"] = "adam"
    loss_function: Literal["ctc", "contrastive_loss", "cross_entropy", "bce", "ctc+discriminator",
                           "combined_ctc"] = "ctc"
    ctc_loss_reduction: Literal["sum", "mean"] = "mean"
    experiment_name: str = "experiment_1"
    experiment_type: str = Field("b2t_wav2vec_sharedaggregation")
    log_every_n_batches: int = 10
    scheduler: Literal["step"] = "step"
    scheduler_step_size: int = 10
    scheduler_gamma: float = 0.1
    return_best_model: bool = True
    best_model_metric: str = Field("loss")
    minimize_best_model_metric: bool = Field(True)
    use_wandb: bool = False
    from_checkpoint: Optional[str] = Field(None, description="(optional) Path to model checkpoint")
    only_test: bool = Field(False)
    predict_on_train: bool = Field(False)
    gradient_clipping: Optional[float] = None
    weight_decay: float = 0.0
    visualize_predictions_n_batches: int = 1
    use_fast_tokenizer: bool = False
    use_prefix_beam_search: bool = True
    beam_search_language_model: str = "openai-community/gpt2"
    whiteNoiseSD: float = 0.0
    constantOffsetSD: float = 0.0
    seed: int = 42
    optimizer_epsilon: float = 1e-8
    early_stopping_patience: Optional[int] = Field(None)
    early_stopping_delta: float = Field(0.0001)
    train_on_val_once: bool = Field(False)
    log_results_as_artifact: bool = False
    results_subdir_name: Optional[str] = None
