"""MI355X-native (gfx950 / CDNA4) b2p2t_gru+w2v training step, a drop-in for the model, experiment
and trainer API of yuanhao-chen-nyoeghau/Wav2Vec2ForBrain (reference `src/`).

Layout mirrors the reference package: model/, datasets/, experiments/, train/, util/, args/.
Compute runs in the hand-written HIP kernels of libb2p_hip.so (csrc/, C ABI in include/b2p_hip.h)
through functional.py.
"""
__version__ = "0.1.0"
