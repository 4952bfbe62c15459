"""config.yaml of a run (reference src/args/yaml_config.py:8-62): cache/result directories, the
dataset split directory, LM paths and W&B settings. The reference writes a template and exits when
the file is missing; here a missing file falls back to a local cache directory (results go to
./cache, data to the synthetic dataset), so `run.py` works out of the box offline."""
from __future__ import annotations

import os
from typing import Optional

import yaml
from pydantic import BaseModel, Field


class YamlConfigModel(BaseModel):
    cache_dir: str = Field(default="cache", description="Directory to store larger temporary files like model "
                                                        "checkpoints in")
    fig_dir: str = Field(default="figures", description="Directory to store figures in")
    n3gram_lm_model_path: str = Field(default="", description="Path to the 3-gram language model")
    n5gram_lm_model_path: str = Field(default="", description="Path to the 5-gram language model")
    dataset_splits_dir: str = Field(default="", description="Directory containing the original train and test "
                                                            "split folder")
    wandb_api_key: str = Field(default="", description="Your Weights and Biases API key.")
    wandb_project_name: str = Field(default="brain2text", description="Your W&B project name.")
    wandb_entity: str = Field(default="machine-learning-hpi", description="Your W&B entity name.")
    timit_dataset_splits_dir: str = Field(default="", description="TIMIT split directory")
    elevenlabs_api_key: Optional[str] = Field(default=None, description="Elevenlabs API key (analysis only)")
    latent_analysis_working_dir: str = Field(default="latent_analysis")


class YamlConfig:
    def __init__(self, config_path: str = "config.yaml"):
        self.config_path = config_path
        self.config = self._load_config()

    def _load_config(self) -> YamlConfigModel:
        if not os.path.exists(self.config_path):
            return YamlConfigModel()
        with open(self.config_path) as f:
            content = yaml.safe_load(f) or {}
        try:
            return YamlConfigModel(**content)
        except Exception as e:
            raise Exception(f"Error validating fields in config file {self.config_path}: \n{e}")
