"""Named workloads of the b2p2t_gru+w2v training step: the BASELINE.json configurations as model
architecture + synthetic batch, and the construction of the build's model for them
with the deterministic portable-PRNG weights (util/init.py) that the golden fixtures were generated
with. Used by bench.py, __graft_entry__ and the tests (tests/helpers.py re-exports these).

The hub is unreachable here, so architectures are restated (model/w2v_config.py) and weights are
random-init of that architecture, as BASELINE.md's synthetic-data rule asks.
"""
from __future__ import annotations

import torch


def bench_config(kind: str = "base", bs: int = 32, L: int = 1024) -> dict:
    """Per-GPU workload of a BASELINE config:
    base      configs[1]: wav2vec2-base (768/12L/12H/3072), GRU H256x2, fc []
    conformer configs[2] (and configs[4] per GPU): wav2vec2-conformer-rope-large (1024/24L/16H/4096,
              k31), README brain encoder H512x3, fc [256]
    large     configs[3] per GPU: wav2vec2-large-960h (1024/24L/16H/4096, post-LN forced by the
              reference), GRU H256x2, fc [] (the 512 -> 1024 projection)"""
    common = dict(seed=42, B=bs, L=L, in_lens=[L] * bs, tgt_range=(60, 120), pos_k=128, pos_groups=16,
                  bidirectional=True, learnable_h0=False, full_grad_max=0, infeasible=False)
    if kind == "conformer":
        return dict(common, name="bench_conformer", hidden_size=1024, layers=24, heads=16, ffn=4096, gru_hidden=512,
                    gru_layers=3, fc_hidden=[256], conformer=True, dw_kernel=31)
    if kind == "large":
        return dict(common, name="bench_large960", hidden_size=1024, layers=24, heads=16, ffn=4096, gru_hidden=256,
                    gru_layers=2, fc_hidden=[])
    if kind != "base":
        raise ValueError(f"unknown workload {kind!r}")
    return dict(common, name="bench_base", hidden_size=768, layers=12, heads=12, ffn=3072, gru_hidden=256,
                gru_layers=2, fc_hidden=[])


def make_batch(cfg):
    """Synthetic inputs: x ~ N(0,1) (B,L,256); day ~ U{0..23}; targets ~ U{4..31}
    padded with 0; data seed 0."""
    g = torch.Generator().manual_seed(0)
    B, L = cfg["B"], cfg["L"]
    x = torch.randn(B, L, 256, generator=g)
    for b, il in enumerate(cfg["in_lens"]):
        x[b, il:] = 0.0   # zero-padded tail like the collate function
    day = torch.randint(0, 24, (B,), generator=g)
    lo, hi = cfg["tgt_range"]
    tl = torch.randint(lo, hi + 1, (B,), generator=g)
    S = int(tl.max())
    tgt = torch.zeros(B, S, dtype=torch.int64)
    for b in range(B):
        tgt[b, :tl[b]] = torch.randint(4, 32, (int(tl[b]),), generator=g)
    if cfg.get("infeasible"):
        # sample 0: more labels (all equal -> needs 2 frames each) than logit frames
        T = (cfg["in_lens"][0] - 32) // 4
        n = min(S, T // 2 + 2)
        tgt[0, :n] = 7
        tl[0] = n
    in_lens = torch.tensor(cfg["in_lens"], dtype=torch.int64)
    return x, day, in_lens, tgt, tl.to(torch.int64)


def w2v_cfg(cfg, train_dropouts=False):
    """The encoder architecture of a workload; train_dropouts: the checkpoints' 0.1 dropouts and
    LayerDrop (train mode as the reference runs it), else all 0 (deterministic parity mode)."""
    from .model.w2v_config import W2VConfig
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
    """The build's W2VBrainEncoderModel / W2VConformerBrainEncoderModel for a workload, with the
    deterministic weights (util.init.init_deterministic_)."""
    from .args import base_args
    from .model import brain_feature_extractor as bfe
    from .model.w2v_custom_feat_extractor import W2VBrainEncoderModel, W2VBrainEncoderModelArgs
    from .util.init import init_deterministic_
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
        from .model.w2v_conformer_custom_feat_extractor import W2VConformerBrainEncoderModel
        model = W2VConformerBrainEncoderModel(brain, name, w2v_config_override=w2v_cfg(cfg, train_dropouts))
    else:
        model = W2VBrainEncoderModel(W2VBrainEncoderModelArgs(w2v_do_stable_layer_norm=cfg.get("stable", False)),
                                     brain, name, skip_loading_weights=True,
                                     w2v_config_override=w2v_cfg(cfg, train_dropouts))
    init_deterministic_(model, cfg["seed"] if seed is None else seed)
    return model.to(device)


class SyntheticStepExperiment:
    """The part of the Experiment API (reference src/experiments/experiment.py:31-171) that the
    Trainer's step reads — base_config, model, create_optimizer, get_scheduler — for a workload model
    without a dataset on disk (bench.py, tests). create_optimizer restates the experiments' param
    groups (b2t_gru_w2v_experiment.py:109-145, b2t_gru_w2v_conformer_experiment.py:87-123):
    unfreeze="brain_encoder" optimises the brain encoder only; "brain_encoder+w2v" adds the w2v
    encoder at w2v_lr (default: lr)."""

    def __init__(self, model, unfreeze: str = "brain_encoder", lr: float = 1e-3, w2v_lr=None,
                 weight_decay: float = 0.0, **config):
        from .args.base_args import BaseExperimentArgsModel
        if unfreeze not in ("brain_encoder", "brain_encoder+w2v"):
            raise ValueError(f"unfreeze strategy {unfreeze!r}")
        self.base_config = BaseExperimentArgsModel(learning_rate=lr, weight_decay=weight_decay, **config)
        self.model = model
        self.unfreeze = unfreeze
        self.w2v_lr = w2v_lr
        self.dataloader_train = self.dataloader_val = self.dataloader_test = None

    def create_optimizer(self):
        from .optim import HipAdam
        groups = [{"params": list(self.model.brain_encoder.parameters())}]
        if self.unfreeze == "brain_encoder+w2v":
            groups.append({"params": list(self.model.w2v_encoder.parameters()),
                           "lr": self.w2v_lr if self.w2v_lr is not None else self.base_config.learning_rate})
        return HipAdam(groups, lr=self.base_config.learning_rate, weight_decay=self.base_config.weight_decay,
                       eps=self.base_config.optimizer_epsilon)

    def get_scheduler(self, optimizer):
        return torch.optim.lr_scheduler.StepLR(optimizer, step_size=self.base_config.scheduler_step_size,
                                               gamma=self.base_config.scheduler_gamma)


def device_batch(cfg, device="cuda"):
    """The workload's synthetic batch as a B2tSampleBatch (on `device`)."""
    from .datasets.batch_types import make_b2t_batch
    x, day, il, tgt, tl = make_batch(cfg)
    b = make_b2t_batch(x, tgt, day, il, tl)
    return b.cuda() if device != "cpu" else b
