"""Build audit (CPU): every hot kernel compiles for gfx950 without scratch (no spills, no
dynamically-indexed private arrays)."""
import pytest


@pytest.mark.parametrize("src", ["gemm.hip", "gemm16.hip", "gru.hip", "elementwise.hip", "ctc.hip"])
def test_no_scratch(src):
    from wav2vec2forbrain_amd.build_lib import audit_scratch
    res = audit_scratch(src)
    assert res, "no kernels found"
    bad = {k: v for k, v in res.items() if v != 0}
    assert not bad, bad
