"""GRU brain-feature encoder — mirrors reference src/model/brain_feature_extractor.py.

BrainFeatureExtractor keeps an nn.GRU and an nn.Sequential of nn.Linear as *parameter
containers* so parameter names, shapes and initialisation match the reference state_dict; the
forward runs each GRU layer through functional.gru_layer (HIP: implicit-Unfold input GEMM for
layer 0, per-step recurrence kernels, BPTT) and the FC stack through functional.linear.
"""
from __future__ import annotations

from typing import Optional

import torch
from pydantic import BaseModel

from .. import functional as Fn
from ..args.base_args import PRETRAINED_LATENT_SIZES
from ..datasets.batch_types import PhonemeSampleBatch, SampleBatch
from ..util.nn_helper import ACTIVATION_FUNCTION, create_fully_connected, run_fully_connected
from .b2p2t_model import B2P2TModel, B2P2TModelArgsModel
from .b2tmodel import B2TModel, ModelOutput


class BrainFeatureExtractorArgsModel(BaseModel):
    encoder_gru_hidden_size: int = 256
    encoder_bidirectional: bool = True
    encoder_num_gru_layers: int = 2
    encoder_bias: bool = True
    encoder_dropout: float = 0.0
    encoder_learnable_inital_state: bool = False
    encoder_fc_hidden_sizes: list[int] = []
    encoder_fc_activation_function: ACTIVATION_FUNCTION = "gelu"


class BrainFeatureExtractor(torch.nn.Module):
    def __init__(self, config: BrainFeatureExtractorArgsModel, in_size, wav2vec_checkpoint: str):
        super().__init__()
        self.config = config
        self.num_directions = 2 if config.encoder_bidirectional else 1
        self.hidden_start = torch.nn.Parameter(
            torch.randn(self.num_directions * config.encoder_num_gru_layers, config.encoder_gru_hidden_size,
                        requires_grad=True))
        self.gru = torch.nn.GRU(in_size, config.encoder_gru_hidden_size, config.encoder_num_gru_layers,
                                dropout=config.encoder_dropout, bias=config.encoder_bias,
                                bidirectional=config.encoder_bidirectional, batch_first=True)
        self.fc = create_fully_connected(config.encoder_gru_hidden_size * self.num_directions,
                                         PRETRAINED_LATENT_SIZES[wav2vec_checkpoint], config.encoder_fc_hidden_sizes,
                                         config.encoder_fc_activation_function)

    def _layer_weights(self, layer: int):
        ws = []
        for sfx in ([""] if self.num_directions == 1 else ["", "_reverse"]):
            g = self.gru
            ws += [getattr(g, f"weight_ih_l{layer}{sfx}"), getattr(g, f"weight_hh_l{layer}{sfx}"),
                   getattr(g, f"bias_ih_l{layer}{sfx}") if g.bias else None,
                   getattr(g, f"bias_hh_l{layer}{sfx}") if g.bias else None]
        return ws

    def forward(self, batch: PhonemeSampleBatch) -> torch.Tensor:
        x, _ = batch
        batch_size = x.shape[0]
        H = self.config.encoder_gru_hidden_size
        nd = self.num_directions
        h0_all = (self.hidden_start.unsqueeze(1).repeat(1, batch_size, 1)
                  if self.config.encoder_learnable_inital_state else None)
        out = x
        nl = self.config.encoder_num_gru_layers
        for layer in range(nl):
            h0 = h0_all[layer * nd:(layer + 1) * nd].contiguous() if h0_all is not None else None
            out = Fn.gru_layer(out, H, nd, self._layer_weights(layer), h0)
            if layer + 1 < nl:
                out = Fn.dropout(out, self.config.encoder_dropout, self.training)
        return run_fully_connected(self.fc, out)


class B2TBrainFeatureExtractor(B2TModel):
    def __init__(self, config: BrainFeatureExtractorArgsModel, wav2vec_checkpoint: str, in_size: int):
        super().__init__()
        self.encoder = BrainFeatureExtractor(config, in_size, wav2vec_checkpoint)

    def forward(self, batch: SampleBatch) -> ModelOutput:
        out = self.encoder(batch)
        return ModelOutput(logits=out, metrics={})


class B2P2TBrainFeatureExtractorArgsModel(BrainFeatureExtractorArgsModel, B2P2TModelArgsModel):
    pass


def bfe_w_preprocessing_from_config(config: B2P2TBrainFeatureExtractorArgsModel, brain_encoder_path: Optional[str],
                                    wav2vec_checkpoint: str):
    """Reference :96-123 (weights-only load, drops discriminator / suc_for_ctc keys, strict)."""
    brain_feat_extractor = B2P2TModel(
        config,
        B2TBrainFeatureExtractor(config, wav2vec_checkpoint,
                                 B2P2TModel.get_in_size_after_preprocessing(config.unfolder_kernel_len)),
    ).cuda()
    if brain_encoder_path is not None:
        state = torch.load(brain_encoder_path, map_location="cuda", weights_only=True)
        for key in [k for k in state.keys() if k.startswith("neural_decoder.discriminator")
                    or k.startswith("neural_decoder.suc_for_ctc")]:
            del state[key]
        brain_feat_extractor.load_state_dict(state, strict=True)
    return brain_feat_extractor
