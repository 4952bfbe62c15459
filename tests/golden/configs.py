"""Fixture configurations shared by make_golden.py (reference side) and the tests (build side)."""
from __future__ import annotations

import torch

CONFIGS = [
    # tiny: every code path, full gradients stored
    dict(name="tiny_a", seed=42, B=3, L=96, in_lens=[96, 80, 64], tgt_range=(2, 8), hidden_size=64, layers=2,
         heads=4, ffn=128, pos_k=16, pos_groups=4, gru_hidden=32, gru_layers=2, bidirectional=True, fc_hidden=[],
         learnable_h0=False, full_grad_max=65536, infeasible=False),
    # tiny variant: 3 GRU layers, fc hidden + GELU, learnable h0, one infeasible sample (zero_infinity)
    dict(name="tiny_b", seed=43, B=2, L=128, in_lens=[128, 128], tgt_range=(3, 9), hidden_size=48, layers=1,
         heads=3, ffn=96, pos_k=8, pos_groups=2, gru_hidden=16, gru_layers=3, bidirectional=True, fc_hidden=[40],
         learnable_h0=True, full_grad_max=65536, infeasible=True),
    # config (1) of BASELINE.json: wav2vec2-base architecture, bs=2, 512-step windows (plumbing case)
    dict(name="plumbing_base", seed=42, B=2, L=512, in_lens=[512, 384], tgt_range=(20, 50), hidden_size=768,
         layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2, bidirectional=True,
         fc_hidden=[], learnable_h0=False, full_grad_max=4096, infeasible=False),
    # Conformer (rotary) tiny: every conformer code path, full small gradients
    dict(name="tiny_conf", seed=44, B=2, L=96, in_lens=[96, 88], tgt_range=(2, 8), hidden_size=64, layers=2,
         heads=4, ffn=128, pos_k=16, pos_groups=4, gru_hidden=32, gru_layers=2, bidirectional=True, fc_hidden=[48],
         learnable_h0=False, full_grad_max=65536, infeasible=False, conformer=True, dw_kernel=7),
    # BASELINE configs[2] architecture (wav2vec2-conformer-rope-large: 1024/24L/16H/4096, k31; README brain
    # encoder H512x3, fc [256]) at bs=2, 288-bin windows
    dict(name="conformer_large_b2", seed=45, B=2, L=288, in_lens=[288, 256], tgt_range=(10, 25), hidden_size=1024,
         layers=24, heads=16, ffn=4096, pos_k=128, pos_groups=16, gru_hidden=512, gru_layers=3, bidirectional=True,
         fc_hidden=[256], learnable_h0=False, full_grad_max=4096, infeasible=False, conformer=True, dw_kernel=31),
    # w2v_do_stable_layer_norm=True (pre-LN encoder, TF Wav2Vec2EncoderStableLayerNorm): tiny and base-size
    dict(name="tiny_stable", seed=46, B=3, L=96, in_lens=[96, 88, 72], tgt_range=(2, 8), hidden_size=64, layers=2,
         heads=4, ffn=128, pos_k=16, pos_groups=4, gru_hidden=32, gru_layers=2, bidirectional=True, fc_hidden=[],
         learnable_h0=False, full_grad_max=65536, infeasible=False, stable=True),
    dict(name="plumbing_stable", seed=47, B=2, L=512, in_lens=[512, 448], tgt_range=(20, 50), hidden_size=768,
         layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2, bidirectional=True,
         fc_hidden=[], learnable_h0=False, full_grad_max=4096, infeasible=False, stable=True),
    # the bench workloads themselves (BASELINE configs[1] and configs[2]) at bs=32, 1024-bin windows:
    # loss, per-parameter gradient norms and sampled gradient entries (inputs are regenerated from the
    # seed, not stored: x alone would be 33 MB)
    dict(name="base_bs32", seed=42, B=32, L=1024, in_lens=[1024] * 32, tgt_range=(60, 120), hidden_size=768,
         layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2, bidirectional=True,
         fc_hidden=[], learnable_h0=False, full_grad_max=0, infeasible=False, big=True),
    dict(name="conformer_large_bs32", seed=42, B=32, L=1024, in_lens=[1024] * 32, tgt_range=(60, 120),
         hidden_size=1024, layers=24, heads=16, ffn=4096, pos_k=128, pos_groups=16, gru_hidden=512, gru_layers=3,
         bidirectional=True, fc_hidden=[256], learnable_h0=False, full_grad_max=0, infeasible=False, conformer=True,
         dw_kernel=31, big=True),
]


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
