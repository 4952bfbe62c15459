"""Pretrained wav2vec2 / wav2vec2-conformer weights from a local HF checkpoint directory.

The reference loads them with `Wav2Vec2WithoutFeatExtrForCTC.from_pretrained(wav2vec_checkpoint)`
(src/model/w2v_custom_feat_extractor.py:43-51) and `Wav2Vec2ConformerWithoutFeatExtrForCTC.from_pretrained`
(src/model/w2v_conformer_custom_feat_extractor.py:24-33): transformers builds a Wav2Vec2ForCTC, swaps
in the encoder-only model, and copies every checkpoint tensor whose key exists in that module tree.
Keys of the audio front end (`feature_extractor.*`, `feature_projection.*`, `masked_spec_embed`,
quantizer / adapter heads) have no counterpart there and are dropped.

Positional-conv weight norm: HF checkpoints store it as `...pos_conv_embed.conv.weight_g/weight_v`,
while the module built under torch >= 2.1 names it `parametrizations.weight.original0/original1`.
transformers 4.35.2 (the reference's pin) did not rename them, so in the authors' runs these two
tensors stayed randomly initialised (src/analysis/latent_analysis_leon.ipynb cell 9: "newly
initialized"). `pos_conv="reference"` (default) reproduces that; `pos_conv="load"` maps g -> original0,
v -> original1 (what later transformers releases do).

The hub is unreachable here: `path` must be a local directory (or file) holding model.safetensors or
pytorch_model.bin. Only non-executing loaders are used (safetensors, torch.load(weights_only=True)).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

_DROP_PREFIXES = ("feature_extractor.", "feature_projection.", "masked_spec_embed", "quantizer.", "project_q.",
                  "project_hid.", "adapter.")


def read_hf_state(path: str) -> Dict[str, torch.Tensor]:
    """Tensors of a local HF checkpoint (directory with model.safetensors / pytorch_model.bin, or
    that file itself)."""
    if os.path.isdir(path):
        for name in ("model.safetensors", "pytorch_model.bin"):
            f = os.path.join(path, name)
            if os.path.exists(f):
                path = f
                break
        else:
            raise FileNotFoundError(f"{path}: no model.safetensors or pytorch_model.bin")
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return dict(load_file(path, device="cpu"))
    return dict(torch.load(path, map_location="cpu", weights_only=True))


def map_hf_keys(hf: Dict[str, torch.Tensor], target_keys, pos_conv: str = "reference"
                ) -> Tuple[Dict[str, torch.Tensor], dict]:
    """HF ForCTC keys -> keys of the build's w2v_encoder module (Wav2Vec2WithoutFeatExtrForCTC or the
    Conformer variant: `wav2vec2.encoder.*` / `wav2vec2_conformer.encoder.*` and `lm_head.*`).
    Returns (state, report) with report = {loaded, dropped, missing, pos_conv}."""
    if pos_conv not in ("reference", "load"):
        raise ValueError("pos_conv must be 'reference' (transformers 4.35.2 behaviour) or 'load'")
    target = set(target_keys)
    out, dropped = {}, []
    for k, v in hf.items():
        kk = k
        if kk.endswith("pos_conv_embed.conv.weight_g") or kk.endswith("pos_conv_embed.conv.weight_v"):
            if pos_conv == "reference":
                dropped.append(k)
                continue
            kk = kk[:-len("weight_g")] + ("parametrizations.weight.original0" if kk.endswith("weight_g")
                                          else "parametrizations.weight.original1")
        if kk not in target:
            dropped.append(k)
            continue
        out[kk] = v
    missing = sorted(target - set(out))
    return out, dict(loaded=len(out), dropped=sorted(dropped), missing=missing, pos_conv=pos_conv)


def load_pretrained_w2v(w2v_encoder: torch.nn.Module, path: str, pos_conv: str = "reference",
                        strict: bool = True) -> dict:
    """Copy a local HF checkpoint into the build's w2v_encoder module (in place, any device).
    strict: every parameter except the positional-conv weight-norm pair (pos_conv='reference') and
    the never-used Conformer `pos_conv_embed` must be present in the checkpoint."""
    own = w2v_encoder.state_dict()
    state, rep = map_hf_keys(read_hf_state(path), own.keys(), pos_conv)
    for k, v in state.items():
        if tuple(own[k].shape) != tuple(v.shape):
            raise ValueError(f"{k}: checkpoint shape {tuple(v.shape)} != model shape {tuple(own[k].shape)}")
    allowed: Optional[tuple] = ("parametrizations.weight.original0", "parametrizations.weight.original1",
                                "running_mean", "running_var", "num_batches_tracked")
    hard = [k for k in rep["missing"] if not k.endswith(allowed) and ".pos_conv_embed." not in k]
    if strict and hard:
        raise KeyError(f"checkpoint {path} lacks {len(hard)} parameters, e.g. {hard[:5]}")
    w2v_encoder.load_state_dict(state, strict=False)
    if hasattr(w2v_encoder, "modules"):
        from .. import functional as Fn
        Fn.bump_param_epoch(list(w2v_encoder.parameters()))   # cached 16-bit weight copies are stale now
    return rep
