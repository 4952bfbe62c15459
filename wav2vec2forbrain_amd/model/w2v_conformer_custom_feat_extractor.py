"""Wav2Vec2-Conformer (rotary) encoder + CTC head — mirrors reference
src/model/w2v_conformer_custom_feat_extractor.py and the transformers modules it instantiates
(Wav2Vec2ConformerEncoder / EncoderLayer / SelfAttention / ConvolutionModule / FeedForward /
RotaryPositionalEmbedding, transformers 4.35.2 semantics).

Parameter names reproduce the reference state_dict
(`w2v_encoder.wav2vec2_conformer.encoder.layers.N.ffn1.intermediate_dense.weight`, ...,
`conv_module.batch_norm.running_mean`, `encoder.embed_positions.inv_freq`, the constructed-but-
unused `encoder.pos_conv_embed.*`, `w2v_encoder.lm_head.*`). The math runs in
functional.{conformer_ffn, conformer_attention, conformer_conv_module, layer_norm} (HIP).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .. import functional as Fn
from ..datasets.batch_types import B2tSampleBatch
from . import w2v_config
from .b2tmodel import B2TModel, ModelOutput
from .w2v_custom_feat_extractor import Wav2Vec2PositionalConvEmbedding


class Wav2Vec2ConformerFeedForward(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.intermediate_dense = nn.Linear(config.hidden_size, config.intermediate_size)
        self.output_dense = nn.Linear(config.intermediate_size, config.hidden_size)


class Wav2Vec2ConformerSelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        if config.position_embeddings_type not in ("rotary", None):
            raise NotImplementedError(f"position_embeddings_type={config.position_embeddings_type!r}: only the "
                                      "rotary (RoPE) conformer used by the reference checkpoint is built")
        self.head_size = config.hidden_size // config.num_attention_heads
        self.num_heads = config.num_attention_heads
        self.linear_q = nn.Linear(config.hidden_size, config.hidden_size)
        self.linear_k = nn.Linear(config.hidden_size, config.hidden_size)
        self.linear_v = nn.Linear(config.hidden_size, config.hidden_size)
        self.linear_out = nn.Linear(config.hidden_size, config.hidden_size)


class Wav2Vec2ConformerConvolutionModule(nn.Module):
    def __init__(self, config):
        super().__init__()
        if (config.conv_depthwise_kernel_size - 1) % 2 == 1:
            raise ValueError("`config.conv_depthwise_kernel_size` should be a odd number for 'SAME' padding")
        d = config.hidden_size
        self.layer_norm = nn.LayerNorm(d)
        self.pointwise_conv1 = nn.Conv1d(d, 2 * d, kernel_size=1, stride=1, padding=0, bias=False)
        self.depthwise_conv = nn.Conv1d(d, d, config.conv_depthwise_kernel_size, stride=1,
                                        padding=(config.conv_depthwise_kernel_size - 1) // 2, groups=d, bias=False)
        self.batch_norm = nn.BatchNorm1d(d)
        self.pointwise_conv2 = nn.Conv1d(d, d, kernel_size=1, stride=1, padding=0, bias=False)


class Wav2Vec2ConformerEncoderLayer(nn.Module):
    """TF conf EncoderLayer.forward: x += .5 FFN1(LN x); x += Attn(LN x); x += Conv(x);
    x += .5 FFN2(LN x); x = LN(x)."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        d = config.hidden_size
        self.ffn1_layer_norm = nn.LayerNorm(d)
        self.ffn1 = Wav2Vec2ConformerFeedForward(config)
        self.self_attn_layer_norm = nn.LayerNorm(d)
        self.self_attn = Wav2Vec2ConformerSelfAttention(config)
        self.conv_module = Wav2Vec2ConformerConvolutionModule(config)
        self.ffn2_layer_norm = nn.LayerNorm(d)
        self.ffn2 = Wav2Vec2ConformerFeedForward(config)
        self.final_layer_norm = nn.LayerNorm(d)

    def forward(self, x):
        c = self.config
        act = Fn.ACT[{"swish": "silu"}.get(c.hidden_act, c.hidden_act)]
        tr = self.training
        x = Fn.conformer_ffn(x, self.ffn1_layer_norm, self.ffn1.intermediate_dense.weight,
                             self.ffn1.intermediate_dense.bias, self.ffn1.output_dense.weight, self.ffn1.output_dense.bias,
                             act, c.activation_dropout, c.hidden_dropout, tr)
        sa = self.self_attn
        rot = c.rotary_embedding_base if c.position_embeddings_type == "rotary" else None
        # self_attn_dropout uses config.attention_dropout (TF conf EncoderLayer.__init__)
        x = Fn.conformer_attention(x, self.self_attn_layer_norm, sa.linear_q, sa.linear_k, sa.linear_v, sa.linear_out,
                                   sa.num_heads, rot, c.attention_dropout, c.attention_dropout, tr)
        x = Fn.conformer_conv_module(x, self.conv_module, act, c.conformer_conv_dropout, tr)
        x = Fn.conformer_ffn(x, self.ffn2_layer_norm, self.ffn2.intermediate_dense.weight,
                             self.ffn2.intermediate_dense.bias, self.ffn2.output_dense.weight, self.ffn2.output_dense.bias,
                             act, c.activation_dropout, c.hidden_dropout, tr)
        return Fn.layer_norm(x, self.final_layer_norm.weight, self.final_layer_norm.bias, self.final_layer_norm.eps)


class Wav2Vec2ConformerRotaryPositionalEmbedding(nn.Module):
    def __init__(self, config):
        super().__init__()
        dim = config.hidden_size // config.num_attention_heads
        inv_freq = 1.0 / (config.rotary_embedding_base ** (torch.arange(0, dim, 2, dtype=torch.int64).float() / dim))
        self.register_buffer("inv_freq", inv_freq)


class Wav2Vec2ConformerEncoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embed_positions = (Wav2Vec2ConformerRotaryPositionalEmbedding(config)
                                if config.position_embeddings_type == "rotary" else None)
        self.pos_conv_embed = Wav2Vec2PositionalConvEmbedding(config)   # constructed, never called (TF conf)
        self.layer_norm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.layers = nn.ModuleList([Wav2Vec2ConformerEncoderLayer(config) for _ in range(config.num_hidden_layers)])

    def forward(self, hidden_states):
        c = self.config
        hidden_states = Fn.dropout(hidden_states, c.hidden_dropout, self.training)
        graph_ld = self.training and c.layerdrop > 0 and Fn.capturing() and Fn.GRAPH_LAYERDROP
        for layer in self.layers:
            dropout_probability = torch.rand([])
            if graph_ld:   # captured step: device-drawn LayerDrop (Fn.layerdrop_layer)
                hidden_states = Fn.layerdrop_layer(layer, hidden_states, c.layerdrop)
                continue
            skip = self.training and bool(dropout_probability < c.layerdrop)
            if not skip:
                hidden_states = layer(hidden_states)
        return Fn.layer_norm(hidden_states, self.layer_norm.weight, self.layer_norm.bias, self.layer_norm.eps)


class Wav2Vec2ConformerWithoutFeatExtrModel(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.encoder = Wav2Vec2ConformerEncoder(config)

    def forward(self, input_values):
        return self.encoder(input_values)


class Wav2Vec2ConformerWithoutFeatExtrForCTC(nn.Module):
    """Reference :62-76: encoder -> dropout(final_dropout) -> lm_head."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.wav2vec2_conformer = Wav2Vec2ConformerWithoutFeatExtrModel(config)
        self.lm_head = nn.Linear(config.hidden_size, config.vocab_size)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, std=config.initializer_range)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        hidden_states = self.wav2vec2_conformer(x)
        hidden_states = Fn.dropout(hidden_states, self.config.final_dropout, self.training)
        return Fn.linear(hidden_states, self.lm_head.weight, self.lm_head.bias)


class W2VConformerBrainEncoderModel(B2TModel):
    """Reference :16-59 (output has no logit_lens, as in the reference)."""

    def __init__(self, brain_encoder: B2TModel, wav2vec_checkpoint: str,
                 w2v_config_override: Optional[w2v_config.W2VConfig] = None):
        super().__init__()
        self.brain_encoder = brain_encoder
        cfg = w2v_config_override if w2v_config_override is not None else w2v_config.from_pretrained(wav2vec_checkpoint)
        if not cfg.conformer:
            cfg.conformer = True
        self.w2v_encoder = Wav2Vec2ConformerWithoutFeatExtrForCTC(cfg)
        if w2v_config_override is None:   # reference :27-33 always loads the checkpoint's weights
            from .w2v_custom_feat_extractor import _load_or_note
            _load_or_note(self.w2v_encoder, wav2vec_checkpoint)
        self.blank = 0
        self.sync_metrics = True
        # bf16 mode: the Conformer's forward GEMMs on fp16 MFMA (Fn.forward_f16: removes the CTC-loss
        # bias of bf16 logit noise over 24 layers; backward stays bf16)
        self.forward_f16 = True
        # data-parallel runs: BatchNorm statistics over the global batch (SyncBN), so a DP step equals
        # the single-process step on the same global batch; False = per-rank stats
        self.sync_batchnorm = True
        self.process_group = None

    def forward(self, batch: B2tSampleBatch):
        # the encoder's attention dropout keep masks drawn on a side stream beside the GRU (Fn.attn_keep_plan)
        with Fn.attn_keep_plan_cfg(self.w2v_encoder.config, self.brain_encoder, batch.input, self.training):
            return self._forward(batch)

    def _forward(self, batch: B2tSampleBatch):
        # the brain encoder's forward GEMMs on fp16 operands too: its GRU features feed every later
        # step's update (bf16 operands there put 3.7e-4 relative into the step-1 loss, tools/traj_err.py)
        with Fn.forward_f16(self.forward_f16):
            encoded_brain = self.brain_encoder.forward(batch)
        targets = batch.target
        assert targets is not None
        targets = Fn.ctc_targets(targets)   # reference: where(targets < 1, -100, targets)
        import torch.distributed as dist
        from ..train.ddp import dp_active
        sync = self.training and self.sync_batchnorm and dp_active(self.process_group)
        with Fn.forward_f16(self.forward_f16), Fn.sync_batchnorm(
                (self.process_group or dist.group.WORLD) if sync else None):
            w2v_output = self.w2v_encoder.forward(encoded_brain.logits)
        ctc_loss = (Fn.ctc_loss(w2v_output, targets, encoded_brain.logit_lens, batch.target_lens, self.blank)
                    if batch.target_lens is not None and encoded_brain.logit_lens is not None else None)
        metrics = {}
        if ctc_loss is not None:
            metrics["ctc_loss"] = Fn.loss_item(ctc_loss) if self.sync_metrics else ctc_loss.detach()
        return ModelOutput(w2v_output, metrics, loss=ctc_loss)
