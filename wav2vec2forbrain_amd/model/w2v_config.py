"""Offline Wav2Vec2 / Wav2Vec2-Conformer configuration (replaces `*Config.from_pretrained(<hub name>)`,
reference src/model/w2v_custom_feat_extractor.py:36-41 and
src/model/w2v_conformer_custom_feat_extractor.py:24-26, which need the Hugging Face hub).

Field names follow transformers' Wav2Vec2Config / Wav2Vec2ConformerConfig. The presets restate the
architecture of the named checkpoints; the hub is unreachable here, so dropout / layerdrop values
of the presets are the published transformers defaults for these checkpoints and are marked
unverifiable offline in DESIGN.md.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field, asdict
from typing import Optional


@dataclass
class W2VConfig:
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout: float = 0.1
    activation_dropout: float = 0.1
    attention_dropout: float = 0.1
    final_dropout: float = 0.1
    layerdrop: float = 0.1
    layer_norm_eps: float = 1e-5
    num_conv_pos_embeddings: int = 128
    num_conv_pos_embedding_groups: int = 16
    vocab_size: int = 32
    do_stable_layer_norm: bool = False
    initializer_range: float = 0.02
    # conformer
    conformer: bool = False
    position_embeddings_type: Optional[str] = None     # "rotary" for the RoPE conformer
    rotary_embedding_base: int = 10000
    conv_depthwise_kernel_size: int = 31
    conformer_conv_dropout: float = 0.1

    def to_dict(self):
        return asdict(self)


_BASE = W2VConfig()
_LARGE = W2VConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)

PRESETS: dict[str, W2VConfig] = {
    "facebook/wav2vec2-base-960h": _BASE,
    "facebook/wav2vec2-base-100h": _BASE,
    # reference configs list "facebook/wav2vec2-base"; it is not a PRETRAINED_LATENT_SIZES key, the
    # architecture is the base one
    "facebook/wav2vec2-base": _BASE,
    "facebook/wav2vec2-large-960h": _LARGE,
    "jonatasgrosman/wav2vec2-large-xlsr-53-english": W2VConfig(
        hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
        do_stable_layer_norm=True, layerdrop=0.05),
    "facebook/wav2vec2-conformer-rope-large-960h-ft": W2VConfig(
        hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096, hidden_act="swish",
        conformer=True, position_embeddings_type="rotary", rotary_embedding_base=10000,
        conv_depthwise_kernel_size=31),
}


def from_local_dir(path: str) -> W2VConfig:
    """Architecture of a local HF checkpoint directory (its config.json: Wav2Vec2Config /
    Wav2Vec2ConformerConfig fields; unknown fields ignored)."""
    import json
    import os
    with open(os.path.join(path, "config.json")) as f:
        js = json.load(f)
    cfg = W2VConfig()
    for k, v in js.items():
        if hasattr(cfg, k) and k != "conformer":
            setattr(cfg, k, v)
    cfg.conformer = "conformer" in str(js.get("model_type", ""))
    return cfg


def from_pretrained(name: str, **overrides) -> W2VConfig:
    import os
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        cfg = from_local_dir(name)
    elif name not in PRESETS:
        raise KeyError(f"no offline preset for {name!r} and no local checkpoint directory; known: {sorted(PRESETS)}")
    else:
        cfg = copy.deepcopy(PRESETS[name])
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise AttributeError(f"W2VConfig has no field {k!r}")
        setattr(cfg, k, v)
    return cfg
