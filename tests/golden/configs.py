"""Fixture configurations shared by make_golden.py (reference side) and the tests (build side)."""
from __future__ import annotations

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
    # the base architecture on 1,280-bin windows (T' = 313 frames: the 512-key fused attention class)
    dict(name="base_L1280", seed=50, B=2, L=1280, in_lens=[1280, 1100], tgt_range=(30, 60), hidden_size=768,
         layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2, bidirectional=True,
         fc_hidden=[], learnable_h0=False, full_grad_max=4096, infeasible=False, long=True),
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
    # seed, not stored: x alone would be 33 MB), and the bench's 3-step Adam trajectory over the brain
    # encoder (bench.py parity: lr 1e-3, frozen w2v)
    dict(name="base_bs32", seed=42, B=32, L=1024, in_lens=[1024] * 32, tgt_range=(60, 120), hidden_size=768,
         layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2, bidirectional=True,
         fc_hidden=[], learnable_h0=False, full_grad_max=0, infeasible=False, big=True,
         adam=dict(steps=3, lr=1e-3, w2v_lr=None, wd=0.0)),
    dict(name="conformer_large_bs32", seed=42, B=32, L=1024, in_lens=[1024] * 32, tgt_range=(60, 120),
         hidden_size=1024, layers=24, heads=16, ffn=4096, pos_k=128, pos_groups=16, gru_hidden=512, gru_layers=3,
         bidirectional=True, fc_hidden=[256], learnable_h0=False, full_grad_max=0, infeasible=False, conformer=True,
         dw_kernel=31, big=True, adam=dict(steps=3, lr=1e-3, w2v_lr=None, wd=0.0)),
    # BASELINE configs[3] per GPU: wav2vec2-large-960h architecture (post-LN forced by the reference,
    # w2v_custom_feat_extractor.py:18-19,36-41: 1024/24L/16H/4096), GRU H256x2, fc [] (the 512 -> 1024
    # projection), 32 samples x 1024 bins; plus 2 Adam steps over the brain encoder (frozen w2v)
    dict(name="large960_bs32", seed=48, B=32, L=1024, in_lens=[1024] * 32, tgt_range=(60, 120), hidden_size=1024,
         layers=24, heads=16, ffn=4096, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2, bidirectional=True,
         fc_hidden=[], learnable_h0=False, full_grad_max=0, infeasible=False, big=True,
         adam=dict(steps=2, lr=1e-3, w2v_lr=None, wd=0.0)),
    # BASELINE configs[4] per GPU (primary reading: global 64 = 8/GPU): Conformer-large with
    # unfreeze_strategy=brain_encoder+w2v (b2t_gru_w2v_conformer_experiment.py:87-123: two param groups,
    # w2v_learning_rate for the encoder), 3 Adam steps with L2 weight decay over all 618 M parameters
    dict(name="conformer_large_ft_bs8", seed=49, B=8, L=1024, in_lens=[1024] * 6 + [896, 768], tgt_range=(60, 120),
         hidden_size=1024, layers=24, heads=16, ffn=4096, pos_k=128, pos_groups=16, gru_hidden=512, gru_layers=3,
         bidirectional=True, fc_hidden=[256], learnable_h0=False, full_grad_max=0, infeasible=False, conformer=True,
         dw_kernel=31, big=True, adam=dict(steps=3, lr=1e-3, w2v_lr=1e-4, wd=1e-5)),
]


def make_batch(cfg):
    """Synthetic inputs; the generator lives in the package (workloads.make_batch) so
    bench.py and the fixtures draw identical batches."""
    from wav2vec2forbrain_amd.workloads import make_batch as _mb
    return _mb(cfg)
