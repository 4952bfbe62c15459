"""Wav2Vec2 encoder (without the audio feature extractor) + CTC head and loss — mirrors reference
src/model/w2v_custom_feat_extractor.py and the transformers modules it instantiates
(Wav2Vec2Encoder / Wav2Vec2EncoderLayer / Wav2Vec2Attention / Wav2Vec2FeedForward /
Wav2Vec2PositionalConvEmbedding, transformers 4.35.2 semantics).

Module and parameter names reproduce the reference state_dict keys
(`w2v_encoder.wav2vec2.encoder.layers.N.attention.q_proj.weight`, ...,
`...pos_conv_embed.conv.parametrizations.weight.original0/1`, `w2v_encoder.lm_head.*`); torch
nn.Linear / nn.LayerNorm / nn.Conv1d are used only as parameter containers. The math runs in
functional.{pos_conv_ln, encoder_layer, dropout, linear, ctc_loss} (HIP).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

import torch
from pydantic import BaseModel
from torch import nn

from .. import functional as Fn
from ..datasets.batch_types import B2tSampleBatch, PhonemeSampleBatch
from . import w2v_config
from .b2tmodel import B2TModel, ModelOutput


class W2VBrainEncoderModelArgs(BaseModel):
    w2v_do_stable_layer_norm: bool = False


# ------------------------------------------------------------------ parameter containers (HF names)
class Wav2Vec2Attention(nn.Module):
    def __init__(self, embed_dim: int, num_heads: int):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.out_proj = nn.Linear(embed_dim, embed_dim)


class Wav2Vec2FeedForward(nn.Module):
    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__()
        self.intermediate_dense = nn.Linear(config.hidden_size, config.intermediate_size)
        self.output_dense = nn.Linear(config.intermediate_size, config.hidden_size)


class Wav2Vec2EncoderLayer(nn.Module):
    """Post-LN layer (TF Wav2Vec2EncoderLayer.forward): x = LN(x + drop(Attn(x))); x = LN(x + FFN(x))."""

    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__()
        self.config = config
        self.attention = Wav2Vec2Attention(config.hidden_size, config.num_attention_heads)
        self.layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.feed_forward = Wav2Vec2FeedForward(config)
        self.final_layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)

    def params(self):
        a, f = self.attention, self.feed_forward
        return (a.q_proj.weight, a.q_proj.bias, a.k_proj.weight, a.k_proj.bias, a.v_proj.weight, a.v_proj.bias,
                a.out_proj.weight, a.out_proj.bias, self.layer_norm.weight, self.layer_norm.bias,
                f.intermediate_dense.weight, f.intermediate_dense.bias, f.output_dense.weight, f.output_dense.bias,
                self.final_layer_norm.weight, self.final_layer_norm.bias)

    def forward(self, hidden_states):
        c = self.config
        if c.hidden_act not in ("gelu",):
            raise NotImplementedError(f"hidden_act {c.hidden_act!r} for the wav2vec2 encoder layer")
        return Fn.encoder_layer(hidden_states, self.params(), c.num_attention_heads, c.layer_norm_eps,
                                c.attention_dropout, c.hidden_dropout, c.activation_dropout, self.training)


class Wav2Vec2EncoderLayerStableLayerNorm(Wav2Vec2EncoderLayer):
    """Pre-LN layer (TF Wav2Vec2EncoderLayerStableLayerNorm.forward), same parameters and names:
    x = x + drop(Attn(LN(x))); x = x + FFN(final_LN(x)), FFN = drop(W2 drop(GELU(W1 x + b1)) + b2).
    Runs on the pre-LN blocks the Conformer uses (functional.conformer_attention without rotary,
    functional.conformer_ffn with a full residual step)."""

    def forward(self, hidden_states):
        c = self.config
        if c.hidden_act not in ("gelu",):
            raise NotImplementedError(f"hidden_act {c.hidden_act!r} for the wav2vec2 encoder layer")
        a, f = self.attention, self.feed_forward
        x = Fn.conformer_attention(hidden_states, self.layer_norm, a.q_proj, a.k_proj, a.v_proj, a.out_proj,
                                   c.num_attention_heads, None, c.attention_dropout, c.hidden_dropout, self.training)
        return Fn.conformer_ffn(x, self.final_layer_norm, f.intermediate_dense.weight, f.intermediate_dense.bias,
                                f.output_dense.weight, f.output_dense.bias, Fn.ACT["gelu"], c.activation_dropout,
                                c.hidden_dropout, self.training, scale=1.0)


class Wav2Vec2PositionalConvEmbedding(nn.Module):
    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__()
        k = config.num_conv_pos_embeddings
        conv = nn.Conv1d(config.hidden_size, config.hidden_size, kernel_size=k, padding=k // 2,
                         groups=config.num_conv_pos_embedding_groups)
        nn.init.normal_(conv.weight, mean=0, std=2 * math.sqrt(1 / (k * config.hidden_size)))
        nn.init.constant_(conv.bias, 0)
        self.conv = nn.utils.parametrizations.weight_norm(conv, name="weight", dim=2)
        self.groups = config.num_conv_pos_embedding_groups
        if k % 2 != 0:
            raise NotImplementedError("odd num_conv_pos_embeddings (no SamePad frame removal) is not wired")

    def weights(self):
        p = self.conv.parametrizations.weight
        return p.original0, p.original1, self.conv.bias


class Wav2Vec2Encoder(nn.Module):
    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__()
        self.config = config
        self.pos_conv_embed = Wav2Vec2PositionalConvEmbedding(config)
        self.layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.layers = nn.ModuleList([Wav2Vec2EncoderLayer(config) for _ in range(config.num_hidden_layers)])

    def forward(self, hidden_states):
        c = self.config
        g, v, cb = self.pos_conv_embed.weights()
        # hidden = dropout(LN(x + gelu(posconv(x))))  (TF Wav2Vec2Encoder.forward)
        hidden_states = Fn.pos_conv_ln(hidden_states, g, v, cb, self.layer_norm.weight, self.layer_norm.bias,
                                       self.pos_conv_embed.groups, c.layer_norm_eps, c.hidden_dropout, self.training)
        graph_ld = self.training and c.layerdrop > 0 and Fn.capturing() and Fn.GRAPH_LAYERDROP
        for layer in self.layers:
            # LayerDrop: one CPU torch.rand([]) draw per layer, as the reference's encoder does; inside
            # a captured step the draw moves to the device (redrawn on every replay)
            dropout_probability = torch.rand([])
            if graph_ld:
                hidden_states = Fn.layerdrop_layer(layer, hidden_states, c.layerdrop)
                continue
            skip_the_layer = self.training and bool(dropout_probability < c.layerdrop)
            if not skip_the_layer:
                hidden_states = layer(hidden_states)
        return hidden_states


class Wav2Vec2EncoderStableLayerNorm(Wav2Vec2Encoder):
    """TF Wav2Vec2EncoderStableLayerNorm.forward (reference :18-19 with w2v_do_stable_layer_norm=True):
    x = dropout(x + gelu(posconv(x))) (no LayerNorm before the layers); pre-LN layers under LayerDrop;
    final LayerNorm after them. Same parameter names as the post-LN encoder."""

    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__(config)
        self.layers = nn.ModuleList([Wav2Vec2EncoderLayerStableLayerNorm(config)
                                     for _ in range(config.num_hidden_layers)])

    def forward(self, hidden_states):
        c = self.config
        g, v, cb = self.pos_conv_embed.weights()
        hidden_states = Fn.pos_conv_ln(hidden_states, g, v, cb, None, None, self.pos_conv_embed.groups,
                                       c.layer_norm_eps, c.hidden_dropout, self.training)
        graph_ld = self.training and c.layerdrop > 0 and Fn.capturing() and Fn.GRAPH_LAYERDROP
        for layer in self.layers:
            dropout_probability = torch.rand([])
            if graph_ld:
                hidden_states = Fn.layerdrop_layer(layer, hidden_states, c.layerdrop)
                continue
            if not (self.training and bool(dropout_probability < c.layerdrop)):
                hidden_states = layer(hidden_states)
        return Fn.layer_norm(hidden_states, self.layer_norm.weight, self.layer_norm.bias, c.layer_norm_eps)


class Wav2Vec2WithoutFeatExtrModel(nn.Module):
    """Reference :156-191 (encoder only, attention_mask=None, no adapter)."""

    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__()
        self.config = config
        # reference :18-19,36-41: do_stable_layer_norm = w2v_do_stable_layer_norm selects the pre-LN encoder
        self.encoder = Wav2Vec2EncoderStableLayerNorm(config) if config.do_stable_layer_norm else Wav2Vec2Encoder(config)

    def forward(self, input_values):
        return self.encoder(input_values)


class Wav2Vec2WithoutFeatExtrForCTC(nn.Module):
    """Reference :139-153: encoder -> dropout(final_dropout) -> lm_head."""

    def __init__(self, config: w2v_config.W2VConfig):
        super().__init__()
        self.config = config
        self.wav2vec2 = Wav2Vec2WithoutFeatExtrModel(config)
        self.lm_head = nn.Linear(config.hidden_size, config.vocab_size)
        nn.init.normal_(self.lm_head.weight, std=config.initializer_range)
        nn.init.zeros_(self.lm_head.bias)
        for m in self.wav2vec2.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, std=config.initializer_range)
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        hidden_states = self.wav2vec2(x)
        hidden_states = Fn.dropout(hidden_states, self.config.final_dropout, self.training)
        logits = Fn.linear(hidden_states, self.lm_head.weight, self.lm_head.bias)
        return logits, hidden_states


# Set while an Experiment builds its model with --from_checkpoint: the whole state dict is loaded
# right after construction, so a hub name that cannot be fetched offline is not an error then.
_WEIGHTS_LOADED_LATER = [False]


class weights_loaded_later:
    def __init__(self, on: bool):
        self.on = bool(on)

    def __enter__(self):
        self.old = _WEIGHTS_LOADED_LATER[0]
        _WEIGHTS_LOADED_LATER[0] = self.on or self.old

    def __exit__(self, *exc):
        _WEIGHTS_LOADED_LATER[0] = self.old


def _load_or_note(w2v_encoder, wav2vec_checkpoint: str) -> None:
    """Reference from_pretrained weight load (:43-51) from a local HF checkpoint directory. The
    reference either loads the pretrained weights or fails; so does this: a hub name (unreachable
    offline) raises, unless the weights come afterwards (--from_checkpoint, weights_loaded_later) or
    the run opts into random-init encoder weights explicitly (B2P_RANDOM_W2V_WEIGHTS=1: synthetic
    benchmarks and tests), instead of silently training against a random frozen encoder."""
    import os
    if os.path.isdir(wav2vec_checkpoint):
        from ..util.hf_weights import load_pretrained_w2v
        rep = load_pretrained_w2v(w2v_encoder, wav2vec_checkpoint)
        print(f"loaded {rep['loaded']} tensors from {wav2vec_checkpoint} (dropped {len(rep['dropped'])}; "
              f"positional-conv weight norm: {rep['pos_conv']})")
    elif _WEIGHTS_LOADED_LATER[0]:
        print(f"Note: {wav2vec_checkpoint} is not a local checkpoint directory; the encoder weights come from "
              "the checkpoint loaded after construction")
    elif os.environ.get("B2P_RANDOM_W2V_WEIGHTS") == "1":
        print(f"Note: B2P_RANDOM_W2V_WEIGHTS=1: the {wav2vec_checkpoint} encoder keeps random-init weights")
    else:
        raise RuntimeError(
            f"pretrained weights for {wav2vec_checkpoint!r} cannot be fetched (no network): pass a local HF "
            "checkpoint directory as --wav2vec_checkpoint, load a full model with --from_checkpoint, set "
            "--w2v_skip_loading_weights true (b2p2t_gru+w2v), or set B2P_RANDOM_W2V_WEIGHTS=1 to train "
            "against random-init encoder weights on purpose")


class W2VBrainEncoderModel(B2TModel):
    """Reference :22-136. `wav2vec_checkpoint` selects an offline architecture preset (the hub is
    unreachable); pretrained weights are loaded through load_state_dict / from_checkpoint."""

    def __init__(self, config: W2VBrainEncoderModelArgs, brain_encoder: B2TModel, wav2vec_checkpoint: str,
                 head: Optional[nn.Module] = None, skip_loading_weights: bool = False,
                 pre_w2v_head_for_additional_loss: Optional[B2TModel] = None,
                 additonal_loss_weight: Optional[float] = None, additional_loss_squared: Optional[bool] = False,
                 w2v_config_override: Optional[w2v_config.W2VConfig] = None):
        super().__init__()
        self.brain_encoder = brain_encoder
        if w2v_config_override is not None:   # explicit architecture; the stable-LN switch still follows the args
            cfg = dataclasses.replace(w2v_config_override, do_stable_layer_norm=config.w2v_do_stable_layer_norm)
        else:
            cfg = w2v_config.from_pretrained(wav2vec_checkpoint, do_stable_layer_norm=config.w2v_do_stable_layer_norm)
        self.w2v_encoder = Wav2Vec2WithoutFeatExtrForCTC(cfg)
        if not skip_loading_weights:
            _load_or_note(self.w2v_encoder, wav2vec_checkpoint)
        if head is not None or pre_w2v_head_for_additional_loss is not None:
            raise NotImplementedError("head / pre_w2v_head_for_additional_loss are not on the b2p2t_gru+w2v path")
        self.head = None
        self.pre_w2v_head_for_additional_loss = None
        self.blank = 0
        self.sync_metrics = True   # reference reads ctc_loss.item() inside forward (:94)
        # bf16 mode: the brain encoder's forward GEMMs (day layer, GRU input projections, FC stack) and
        # GRU recurrences on fp16 operands (Fn.forward_f16; backward stays bf16)
        self.brain_forward_f16 = True
        # ... and the encoder's fp32-operand forward GEMMs (the stable-LN blocks' projections, lm_head):
        # bf16 noise on the logits biases the convex CTC loss (plumbing_stable: -1.4e-3 relative with
        # bf16 stable-LN blocks, tools/fixture_err2.py); the post-LN layers stage their own 16-bit copies
        self.forward_f16 = True

    def forward(self, batch: B2tSampleBatch):
        # the encoder's attention dropout keep masks drawn on a side stream beside the GRU (Fn.attn_keep_plan)
        with Fn.attn_keep_plan_cfg(self.w2v_encoder.config, self.brain_encoder, batch.input, self.training):
            return self._forward(batch)

    def _forward(self, batch: B2tSampleBatch):
        with Fn.forward_f16(self.brain_forward_f16):
            encoded_brain = self.brain_encoder.forward(batch)
        targets = batch.target
        assert targets is not None
        targets = Fn.ctc_targets(targets)   # reference: where(targets < 1, -100, targets)
        with Fn.forward_f16(self.forward_f16):
            w2v_output, hidden_states = self.w2v_encoder.forward(encoded_brain.logits)
        ctc_loss = (
            Fn.ctc_loss(w2v_output, targets, encoded_brain.logit_lens, batch.target_lens, self.blank)
            if batch.target_lens is not None and encoded_brain.logit_lens is not None else None)
        metrics = {}
        if ctc_loss is not None:
            metrics["ctc_loss"] = Fn.loss_item(ctc_loss) if self.sync_metrics else ctc_loss.detach()
        return ModelOutput(w2v_output, metrics, loss=ctc_loss, logit_lens=encoded_brain.logit_lens,
                           hidden_states=hidden_states)
