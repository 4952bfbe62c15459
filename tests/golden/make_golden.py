"""Generates the golden fixtures tests/golden/*.npz by running THE REFERENCE's own model modules
(/root/reference/src/model/*) on CPU, fp32, deterministic mode (all dropout 0, LayerDrop 0).

Runs only in the build container (it reads /root/reference; never on the GPU box). Stubs, as in
SURVEY.md 8(c3): torch .cuda() -> identity; Wav2Vec2Config.from_pretrained(<hub name>) -> an
explicit local config; attention implementation "eager" (transformers 4.35.2 semantics).
Weights come from wav2vec2forbrain_amd.util.init (deterministic by name), so the fixtures store
inputs, outputs and gradients, not weights.

usage: python tests/golden/make_golden.py   (from the repo root)
"""
from __future__ import annotations

import gc
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
from wav2vec2forbrain_amd.util.init import deterministic_state  # noqa: E402
from tests.golden.configs import CONFIGS, make_batch  # noqa: E402


def _import_reference():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    torch.nn.Module.cuda = lambda self, *a, **k: self
    torch.Tensor.cuda = lambda self, *a, **k: self
    import transformers.models.wav2vec2.modeling_wav2vec2 as tfw
    from src.model import brain_feature_extractor as bfe
    from src.model import w2v_custom_feat_extractor as w2v
    from src.args import base_args
    return tfw, bfe, w2v, base_args


def build_reference_model(cfg, tfw, bfe, w2v, base_args):
    name = "golden/" + cfg["name"]
    base_args.PRETRAINED_LATENT_SIZES[name] = cfg["hidden_size"]
    bfe.PRETRAINED_LATENT_SIZES[name] = cfg["hidden_size"]
    hf = tfw.Wav2Vec2Config(
        hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
        intermediate_size=cfg["ffn"], hidden_act="gelu", hidden_dropout=0.0, activation_dropout=0.0,
        attention_dropout=0.0, feat_proj_dropout=0.0, final_dropout=0.0, layerdrop=0.0,
        num_conv_pos_embeddings=cfg["pos_k"], num_conv_pos_embedding_groups=cfg["pos_groups"], vocab_size=32,
        do_stable_layer_norm=False)
    hf._attn_implementation = "eager"

    def fake_from_pretrained(ckpt, **kw):
        c = tfw.Wav2Vec2Config.from_dict(hf.to_dict())
        for k, v in kw.items():
            setattr(c, k, v)
        c._attn_implementation = "eager"
        return c

    w2v.Wav2Vec2Config.from_pretrained = staticmethod(fake_from_pretrained)
    args = bfe.B2P2TBrainFeatureExtractorArgsModel(
        encoder_gru_hidden_size=cfg["gru_hidden"], encoder_num_gru_layers=cfg["gru_layers"],
        encoder_bidirectional=cfg["bidirectional"], encoder_fc_hidden_sizes=cfg["fc_hidden"],
        encoder_learnable_inital_state=cfg["learnable_h0"])
    brain = bfe.bfe_w_preprocessing_from_config(args, None, name)
    model = w2v.W2VBrainEncoderModel(w2v.W2VBrainEncoderModelArgs(w2v_do_stable_layer_norm=cfg.get("stable", False)),
                                     brain, name, None, True)
    return model


def build_reference_conformer(cfg, bfe, base_args):
    import transformers.models.wav2vec2_conformer.modeling_wav2vec2_conformer as tfc
    from src.model import w2v_conformer_custom_feat_extractor as wc
    name = "golden/" + cfg["name"]
    base_args.PRETRAINED_LATENT_SIZES[name] = cfg["hidden_size"]
    bfe.PRETRAINED_LATENT_SIZES[name] = cfg["hidden_size"]
    hf = tfc.Wav2Vec2ConformerConfig(
        hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
        intermediate_size=cfg["ffn"], hidden_act="swish", position_embeddings_type="rotary",
        rotary_embedding_base=10000, conv_depthwise_kernel_size=cfg["dw_kernel"], hidden_dropout=0.0,
        activation_dropout=0.0, attention_dropout=0.0, feat_proj_dropout=0.0, final_dropout=0.0, layerdrop=0.0,
        conformer_conv_dropout=0.0, num_conv_pos_embeddings=cfg["pos_k"],
        num_conv_pos_embedding_groups=cfg["pos_groups"], vocab_size=32)
    hf._attn_implementation = "eager"
    args = bfe.B2P2TBrainFeatureExtractorArgsModel(
        encoder_gru_hidden_size=cfg["gru_hidden"], encoder_num_gru_layers=cfg["gru_layers"],
        encoder_bidirectional=cfg["bidirectional"], encoder_fc_hidden_sizes=cfg["fc_hidden"],
        encoder_learnable_inital_state=cfg["learnable_h0"])
    brain = bfe.bfe_w_preprocessing_from_config(args, None, name)
    # bypass __init__ (it always calls from_pretrained), then use the reference forward
    model = wc.W2VConformerBrainEncoderModel.__new__(wc.W2VConformerBrainEncoderModel)
    torch.nn.Module.__init__(model)
    model.brain_encoder = brain
    model.w2v_encoder = wc.Wav2Vec2ConformerWithoutFeatExtrForCTC(hf)
    model.loss = torch.nn.CTCLoss(blank=0, reduction="mean", zero_infinity=True)
    return model


def adam_trajectory(model, batch, a, loss1):
    """`a["steps"]` updates of the reference's optimizer (torch.optim.Adam with L2 weight decay,
    src/experiments/experiment.py:25-28) over the param groups create_optimizer builds
    (b2t_gru_w2v_experiment.py:109-145 / b2t_gru_w2v_conformer_experiment.py:87-123): the brain
    encoder, plus the w2v encoder at w2v_learning_rate under unfreeze_strategy=brain_encoder+w2v.
    The gradients of the first update are the ones just recorded. Stores the loss before every update
    and, after the last one, the parameter change at the sampled gradient indices."""
    groups = [{"params": list(model.brain_encoder.parameters())}]
    if a["w2v_lr"] is not None:
        groups.append({"params": list(model.w2v_encoder.parameters()), "lr": a["w2v_lr"]})
    opt = torch.optim.Adam(groups, lr=a["lr"], weight_decay=a["wd"], eps=1e-8)
    p0 = {n: p.detach().clone() for n, p in model.named_parameters()}
    losses = [loss1]
    for k in range(a["steps"]):
        if k:
            opt.zero_grad()
            out = model.forward(batch)
            out.loss.backward()
            losses.append(out.loss.item())
            del out
            gc.collect()
        opt.step()
    res = {"adam_losses": np.array(losses, dtype=np.float64)}
    gen = torch.Generator().manual_seed(8)
    for n, p in model.named_parameters():
        flat = (p.detach() - p0[n]).reshape(-1)
        idx = torch.randint(0, flat.numel(), (256,), generator=gen)
        res["didx/" + n] = idx.numpy()
        res["dval/" + n] = flat[idx].numpy()
        res["dnorm/" + n] = np.array(flat.double().norm().item())
    print(f"  adam losses: {losses}")
    return res


def run(cfg, modules):
    tfw, bfe, w2v, base_args = modules
    torch.manual_seed(0)
    if cfg.get("conformer"):
        model = build_reference_conformer(cfg, bfe, base_args)
    else:
        model = build_reference_model(cfg, tfw, bfe, w2v, base_args)
    sd = deterministic_state([(n, p.shape) for n, p in model.named_parameters()], seed=cfg["seed"])
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith(("gaussian_smoother.weight", "inv_freq", "running_mean", "running_var", "num_batches_tracked"))
               for k in missing), missing
    model.train()   # deterministic: every dropout and layerdrop is 0
    from src.datasets.batch_types import B2tSampleBatch
    x, day, in_lens, tgt, tgt_lens = make_batch(cfg)
    batch = B2tSampleBatch(x, tgt)
    batch.day_idxs = day
    batch.input_lens = in_lens
    batch.target_lens = tgt_lens
    out = model.forward(batch)
    out.loss.backward()
    res = {"loss": np.array(out.loss.item(), dtype=np.float64),
           "logits": out.logits.detach().numpy(),
           "day_idxs": day.numpy(), "input_lens": in_lens.numpy(), "target": tgt.numpy(),
           "target_lens": tgt_lens.numpy()}
    if cfg.get("big"):
        # regenerated from the seed by the tests; the checksum pins the generator
        res["x_sum"] = np.array(x.double().sum().item())
        res["x_abs_sum"] = np.array(x.double().abs().sum().item())
    else:
        res["x"] = x.numpy()
    names = []
    gen = torch.Generator().manual_seed(7)
    for n, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        names.append(n)
        res["gnorm/" + n] = np.array(g.double().norm().item())
        flat = g.reshape(-1)
        if flat.numel() <= cfg["full_grad_max"]:
            res["grad/" + n] = g.numpy()
        else:
            idx = torch.randint(0, flat.numel(), (1024,), generator=gen)
            res["gidx/" + n] = idx.numpy()
            res["gval/" + n] = flat[idx].numpy()
    res["param_names"] = np.array(names)
    if out.logit_lens is not None:
        res["logit_lens"] = out.logit_lens.numpy()
    for n, bt in model.named_buffers():
        if "running_" in n:
            # a copy: numpy() shares the buffer's memory, and the Adam trajectory's forwards below
            # update the running statistics in place
            res["buf/" + n] = bt.detach().clone().numpy()
    if cfg.get("adam"):
        loss1 = out.loss.item()
        del out   # the Conformer-large bs=32 trajectory needs the first step's memory back (64 GB host)
        gc.collect()
        res.update(adam_trajectory(model, batch, cfg["adam"], loss1))
        path = os.path.join(OUT, f"{cfg['name']}.npz")
        np.savez_compressed(path, **res)
        print(f"{path}: loss={loss1:.6f}  ({os.path.getsize(path)/1e6:.2f} MB)", flush=True)
        return
    path = os.path.join(OUT, f"{cfg['name']}.npz")
    np.savez_compressed(path, **res)
    print(f"{path}: loss={out.loss.item():.6f}  ({os.path.getsize(path)/1e6:.2f} MB)")


if __name__ == "__main__":
    mods = _import_reference()
    torch.set_num_threads(8)
    only = sys.argv[1:]
    for c in CONFIGS:
        if not only or c["name"] in only:
            run(c, mods)
