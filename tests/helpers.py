"""Shared test helpers: fixture loading, oracle configs, model construction."""
from __future__ import annotations

import os

import numpy as np
import torch

from tests.golden.configs import CONFIGS, make_batch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CFG = {c["name"]: c for c in CONFIGS}


def load_fixture(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def oracle_cfg(cfg):
    from oracle.b2p2t_oracle import OracleConfig, ConformerOracleConfig
    if cfg.get("conformer"):
        return ConformerOracleConfig(
            gru_hidden=cfg["gru_hidden"], gru_layers=cfg["gru_layers"], bidirectional=cfg["bidirectional"],
            fc_hidden_sizes=list(cfg["fc_hidden"]), learnable_initial_state=cfg["learnable_h0"],
            hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
            intermediate_size=cfg["ffn"], num_conv_pos_embeddings=cfg["pos_k"],
            num_conv_pos_embedding_groups=cfg["pos_groups"], conv_depthwise_kernel_size=cfg["dw_kernel"])
    return OracleConfig(gru_hidden=cfg["gru_hidden"], gru_layers=cfg["gru_layers"], bidirectional=cfg["bidirectional"],
                        fc_hidden_sizes=list(cfg["fc_hidden"]), learnable_initial_state=cfg["learnable_h0"],
                        hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["layers"],
                        num_attention_heads=cfg["heads"], intermediate_size=cfg["ffn"],
                        num_conv_pos_embeddings=cfg["pos_k"], num_conv_pos_embedding_groups=cfg["pos_groups"],
                        do_stable_layer_norm=cfg.get("stable", False))


def w2v_cfg(cfg, train_dropouts=False):
    from wav2vec2forbrain_amd.model.w2v_config import W2VConfig
    p = 0.1 if train_dropouts else 0.0
    extra = {}
    if cfg.get("conformer"):
        extra = dict(conformer=True, position_embeddings_type="rotary", hidden_act="swish",
                     conv_depthwise_kernel_size=cfg["dw_kernel"], conformer_conv_dropout=p)
    return W2VConfig(hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
                     intermediate_size=cfg["ffn"], hidden_dropout=p, activation_dropout=p, attention_dropout=p,
                     final_dropout=p, layerdrop=p, num_conv_pos_embeddings=cfg["pos_k"],
                     num_conv_pos_embedding_groups=cfg["pos_groups"], **extra)


def build_model(cfg, device="cuda", seed=None, train_dropouts=False):
    """The build's W2VBrainEncoderModel for a fixture config with the deterministic weights."""
    from wav2vec2forbrain_amd.args import base_args
    from wav2vec2forbrain_amd.model import brain_feature_extractor as bfe
    from wav2vec2forbrain_amd.model.w2v_custom_feat_extractor import W2VBrainEncoderModel, W2VBrainEncoderModelArgs
    from wav2vec2forbrain_amd.util.init import init_deterministic_
    name = "golden/" + cfg["name"]
    base_args.PRETRAINED_LATENT_SIZES[name] = cfg["hidden_size"]
    bfe.PRETRAINED_LATENT_SIZES[name] = cfg["hidden_size"]
    args = bfe.B2P2TBrainFeatureExtractorArgsModel(
        encoder_gru_hidden_size=cfg["gru_hidden"], encoder_num_gru_layers=cfg["gru_layers"],
        encoder_bidirectional=cfg["bidirectional"], encoder_fc_hidden_sizes=list(cfg["fc_hidden"]),
        encoder_learnable_inital_state=cfg["learnable_h0"])
    torch.manual_seed(0)
    brain = bfe.B2P2TModel(args, bfe.B2TBrainFeatureExtractor(args, name, 256 * args.unfolder_kernel_len))
    if cfg.get("conformer"):
        from wav2vec2forbrain_amd.model.w2v_conformer_custom_feat_extractor import W2VConformerBrainEncoderModel
        model = W2VConformerBrainEncoderModel(brain, name, w2v_config_override=w2v_cfg(cfg, train_dropouts))
    else:
        model = W2VBrainEncoderModel(W2VBrainEncoderModelArgs(w2v_do_stable_layer_norm=cfg.get("stable", False)),
                                     brain, name, skip_loading_weights=True,
                                     w2v_config_override=w2v_cfg(cfg, train_dropouts))
    init_deterministic_(model, cfg["seed"] if seed is None else seed)
    return model.to(device)


def oracle_state(cfg):
    from wav2vec2forbrain_amd.util.init import deterministic_state
    model = build_model(cfg, device="cpu")
    return {k: v.detach().clone() for k, v in model.state_dict().items()}


def batch_dict(cfg):
    x, day, in_lens, tgt, tl = make_batch(cfg)
    return dict(x=x, day_idxs=day, input_lens=in_lens, target=tgt, target_lens=tl)
