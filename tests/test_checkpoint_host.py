"""Checkpoint compatibility, host only: pretrained HF wav2vec2 / wav2vec2-conformer
weights from a local checkpoint directory into the build's encoder modules (reference
`from_pretrained`, src/model/w2v_custom_feat_extractor.py:43-51, src/model/w2v_conformer_custom_feat_extractor.py:24-33),
the positional-conv weight-norm key quirk, and model.pt round trips with the reference key names
(src/experiments/experiment.py:70-75, 137-141). The HF checkpoints are written here by transformers
itself (save_pretrained) from small random configs; nothing is downloaded."""
import os

import pytest
import torch

from tests.helpers import CFG, build_model


def _hf_w2v(tmp_path, stable=False):
    import transformers.models.wav2vec2.modeling_wav2vec2 as tfw
    c = tfw.Wav2Vec2Config(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                           num_conv_pos_embeddings=16, num_conv_pos_embedding_groups=4, vocab_size=32,
                           conv_dim=(32, 32), conv_kernel=(3, 3), conv_stride=(2, 2), do_stable_layer_norm=stable)
    torch.manual_seed(3)
    m = tfw.Wav2Vec2ForCTC(c)
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


def _ours_w2v(path):
    from wav2vec2forbrain_amd.model import w2v_config
    from wav2vec2forbrain_amd.model.w2v_custom_feat_extractor import Wav2Vec2WithoutFeatExtrForCTC
    return Wav2Vec2WithoutFeatExtrForCTC(w2v_config.from_pretrained(str(path)))


@pytest.mark.parametrize("stable", [False, True])
def test_hf_w2v_checkpoint_loads_every_encoder_tensor(tmp_path, stable):
    from wav2vec2forbrain_amd.util.hf_weights import load_pretrained_w2v
    hf = _hf_w2v(tmp_path, stable)
    ours = _ours_w2v(tmp_path)
    assert ours.config.do_stable_layer_norm == stable and ours.config.hidden_size == 64
    before = {k: v.clone() for k, v in ours.state_dict().items()}
    rep = load_pretrained_w2v(ours, str(tmp_path), pos_conv="load")
    hsd = hf.state_dict()
    for k, v in ours.state_dict().items():
        assert torch.equal(v, hsd[k]), k
    assert rep["missing"] == []
    assert all(k.startswith(("wav2vec2.feature_extractor.", "wav2vec2.feature_projection.", "wav2vec2.masked_spec_embed"))
               for k in rep["dropped"]), rep["dropped"]
    assert before.keys() == set(hsd) & before.keys()


def test_legacy_weight_norm_keys_are_mapped(tmp_path):
    """Older checkpoints (torch weight_norm): pos_conv_embed.conv.weight_g / weight_v."""
    from wav2vec2forbrain_amd.util.hf_weights import load_pretrained_w2v
    hf = _hf_w2v(tmp_path)
    sd = {}
    for k, v in hf.state_dict().items():
        k = k.replace("parametrizations.weight.original0", "weight_g").replace("parametrizations.weight.original1",
                                                                                "weight_v")
        sd[k] = v
    os.remove(os.path.join(tmp_path, "model.safetensors"))
    torch.save(sd, os.path.join(tmp_path, "pytorch_model.bin"))
    ours = _ours_w2v(tmp_path)
    load_pretrained_w2v(ours, str(tmp_path), pos_conv="load")
    p = ours.wav2vec2.encoder.pos_conv_embed.conv.parametrizations.weight
    assert torch.equal(p.original0, hf.wav2vec2.encoder.pos_conv_embed.conv.parametrizations.weight.original0)
    assert torch.equal(p.original1, hf.wav2vec2.encoder.pos_conv_embed.conv.parametrizations.weight.original1)
    # transformers 4.35.2 (the reference's pin) left this pair at its random initialisation for such
    # checkpoints ("newly initialized", src/analysis/latent_analysis_leon.ipynb cell 9): the default
    ours2 = _ours_w2v(tmp_path)
    init = {k: v.clone() for k, v in ours2.state_dict().items()}
    rep = load_pretrained_w2v(ours2, str(tmp_path))
    assert rep["pos_conv"] == "reference"
    hsd = hf.state_dict()
    for k, v in ours2.state_dict().items():
        assert torch.equal(v, init[k] if k.endswith(("original0", "original1")) else hsd[k]), k


def test_hf_conformer_checkpoint_loads(tmp_path):
    import transformers.models.wav2vec2_conformer.modeling_wav2vec2_conformer as tfc
    from wav2vec2forbrain_amd.model import w2v_config
    from wav2vec2forbrain_amd.model.w2v_conformer_custom_feat_extractor import Wav2Vec2ConformerWithoutFeatExtrForCTC
    from wav2vec2forbrain_amd.util.hf_weights import load_pretrained_w2v
    c = tfc.Wav2Vec2ConformerConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                                    hidden_act="swish", position_embeddings_type="rotary", conv_depthwise_kernel_size=7,
                                    num_conv_pos_embeddings=16, num_conv_pos_embedding_groups=4, vocab_size=32,
                                    conv_dim=(32, 32), conv_kernel=(3, 3), conv_stride=(2, 2))
    torch.manual_seed(4)
    hf = tfc.Wav2Vec2ConformerForCTC(c)
    hf.save_pretrained(tmp_path, safe_serialization=True)
    cfg = w2v_config.from_pretrained(str(tmp_path))
    assert cfg.conformer and cfg.position_embeddings_type == "rotary" and cfg.conv_depthwise_kernel_size == 7
    ours = Wav2Vec2ConformerWithoutFeatExtrForCTC(cfg)
    rep = load_pretrained_w2v(ours, str(tmp_path), pos_conv="load")
    hsd = hf.state_dict()
    for k, v in ours.state_dict().items():
        if k in hsd:
            assert torch.equal(v, hsd[k]), k
    assert not [k for k in rep["missing"] if "pos_conv_embed" not in k and "inv_freq" not in k], rep["missing"]


def test_shape_mismatch_is_an_error(tmp_path):
    from wav2vec2forbrain_amd.model import w2v_config
    from wav2vec2forbrain_amd.model.w2v_custom_feat_extractor import Wav2Vec2WithoutFeatExtrForCTC
    from wav2vec2forbrain_amd.util.hf_weights import load_pretrained_w2v
    _hf_w2v(tmp_path)
    cfg = w2v_config.from_pretrained(str(tmp_path))
    cfg.intermediate_size = 96
    with pytest.raises(ValueError):
        load_pretrained_w2v(Wav2Vec2WithoutFeatExtrForCTC(cfg), str(tmp_path))


@pytest.mark.parametrize("name", ["tiny_a", "tiny_conf"])
def test_model_pt_round_trip_strict(tmp_path, name):
    """store_trained_model's model.pt (reference experiment.py:137-141) loads back strictly into a fresh
    model (from_checkpoint, experiment.py:70-75), tensor for tensor."""
    cfg = CFG[name]
    a = build_model(cfg, device="cpu", seed=1)
    f = os.path.join(tmp_path, "model.pt")
    torch.save(a.state_dict(), f)
    b = build_model(cfg, device="cpu", seed=2)
    assert any(not torch.equal(x, y) for x, y in zip(a.state_dict().values(), b.state_dict().values()))
    b.load_state_dict(torch.load(f, map_location="cpu", weights_only=True), strict=True)
    for (k, x), (k2, y) in zip(a.state_dict().items(), b.state_dict().items()):
        assert k == k2 and torch.equal(x, y), k
    # brain_encoder.pt (b2t_gru_w2v_experiment.py:202-207) = the brain encoder's own state_dict
    fb = os.path.join(tmp_path, "brain_encoder.pt")
    torch.save(a.brain_encoder.state_dict(), fb)
    c = build_model(cfg, device="cpu", seed=3)
    c.brain_encoder.load_state_dict(torch.load(fb, map_location="cpu", weights_only=True), strict=True)
    assert all(torch.equal(x, y) for x, y in zip(a.brain_encoder.state_dict().values(),
                                                 c.brain_encoder.state_dict().values()))


def test_hub_name_without_weights_raises(monkeypatch):
    """The reference's from_pretrained either loads the pretrained encoder or fails: a hub name that
    cannot be fetched offline raises instead of silently leaving a random frozen encoder, unless the
    weights come later (--from_checkpoint) or random-init weights are asked for explicitly."""
    from wav2vec2forbrain_amd.model import w2v_custom_feat_extractor as w
    from wav2vec2forbrain_amd.model.w2v_config import W2VConfig
    monkeypatch.delenv("B2P_RANDOM_W2V_WEIGHTS", raising=False)
    enc = w.Wav2Vec2WithoutFeatExtrForCTC(W2VConfig(hidden_size=32, num_hidden_layers=1, num_attention_heads=2,
                                                    intermediate_size=64, num_conv_pos_embeddings=8,
                                                    num_conv_pos_embedding_groups=2))
    with pytest.raises(RuntimeError, match="cannot be fetched"):
        w._load_or_note(enc, "facebook/wav2vec2-base-960h")
    with w.weights_loaded_later(True):
        w._load_or_note(enc, "facebook/wav2vec2-base-960h")
    monkeypatch.setenv("B2P_RANDOM_W2V_WEIGHTS", "1")
    w._load_or_note(enc, "facebook/wav2vec2-base-960h")
