"""C-ABI boundary checks (CPU): the library builds/loads and exports every entry point that
include/b2p_hip.h declares; the ctypes binding covers the same set; argument validation errors
surface as RuntimeError without touching a device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "b2p_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(b2p_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    assert "b2p_gemm" in names and "b2p_ctc_fwd_bwd" in names and "b2p_gru_fwd" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    from wav2vec2forbrain_amd import _lib
    lib = _lib.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    from wav2vec2forbrain_amd import _lib
    assert sorted(_lib.exported_symbols()) == _declared()


def test_struct_layout_matches_c():
    import numpy as np
    from wav2vec2forbrain_amd import _lib
    out = np.zeros(3, dtype=np.int64)
    _lib.call("b2p_abi_sizes", out.ctypes.data)
    assert list(out) == [ctypes.sizeof(_lib.Operand), ctypes.sizeof(_lib.Epilogue), ctypes.sizeof(_lib.GemmDesc)]
    for cls in (_lib.Operand, _lib.Epilogue, _lib.GemmDesc):
        for name, _ in cls._fields_:
            assert getattr(cls, name).offset % 4 == 0


def test_argument_validation_without_device():
    from wav2vec2forbrain_amd import _lib
    lib = _lib.load()
    assert lib.b2p_version() >= 1
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.nz1, d.nz2 = 4, 4, 4, 1, 1
    rc = lib.b2p_gemm(ctypes.byref(d), None)          # NULL operands -> error, no launch
    assert rc != 0
    assert b"NULL" in lib.b2p_last_error()
    with pytest.raises(RuntimeError):
        _lib.call("b2p_dropout", None, None, 10, 0.5, 1, None)
    assert lib.b2p_ctc_workspace(2, 10, 3, 32) == 2 * (10 * 32 + 2 * 10 * 7)


def test_layerdrop_draw_host_side():
    """LayerDrop device draw (csrc/layerdrop.hip) evaluated on the host: keep rate 1 - p over seeds,
    p = 0 always keeps, and the step counter changes the draw of a fixed seed."""
    from wav2vec2forbrain_amd import functional as Fn
    seeds = range(1, 4001)
    for p in (0.1, 0.5):
        rate = sum(Fn.layerdrop_keep(p, s * 0x9E3779B1) for s in seeds) / len(seeds)
        assert abs(rate - (1 - p)) < 0.03, (p, rate)
    assert all(Fn.layerdrop_keep(0.0, s) for s in range(100))
    draws = {Fn.layerdrop_keep(0.5, 12345, e) for e in range(64)}
    assert draws == {True, False}
    with pytest.raises(RuntimeError):
        Fn.layerdrop_keep(1.0, 1)
