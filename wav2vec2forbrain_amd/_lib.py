"""ctypes binding of libb2p_hip.so (the C ABI declared in include/b2p_hip.h).

This is the binding a maintainer of the reference would add: the reference is Python, so its
"FFI" is ctypes over a C-ABI shared library. torch is imported first so the
HIP runtime it loaded (libamdhip64.so.7) is the one the library binds to; tensors cross the
boundary as raw device pointers and every call is issued on torch's current HIP stream.

There is no fallback: if the library is missing or fails to load, importing the product path
raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede loading the HIP library: shared runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# B2P_LIB_PATH: load another build of the library (A/B of compile-time variants: tools/build_variant.sh)
LIB_PATH = os.environ.get("B2P_LIB_PATH") or os.path.join(_HERE, "libb2p_hip.so")

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_p = ctypes.c_void_p


class Operand(ctypes.Structure):
    _fields_ = [
        ("ptr", c_p), ("ld", c_i64), ("bs1", c_i64), ("bs2", c_i64), ("gather1", c_p),
        ("inner_is_k", c_i32), ("conv", c_i32),
        ("conv_T_out", c_i32), ("conv_T_in", c_i32), ("conv_stride", c_i32), ("conv_pad", c_i32),
        ("conv_Cg", c_i32), ("dtype", c_i32), ("conv_sample_stride", c_i64),
    ]


class Epilogue(ctypes.Structure):
    _fields_ = [
        ("C", c_p), ("ldc", c_i64), ("cbs1", c_i64), ("cbs2", c_i64),
        ("alpha", c_f32), ("beta", c_f32), ("bias", c_p), ("biasbs1", c_i64), ("bias_gather", c_p), ("pre_out", c_p),
        ("act", c_i32), ("act_bwd", c_i32), ("aux", c_p), ("ldaux", c_i64), ("abs1", c_i64),
        ("abs2", c_i64), ("drop_p", c_f32), ("flags", c_i32), ("drop_seed", c_u64),
        ("residual", c_p), ("ldr", c_i64), ("rbs1", c_i64), ("rbs2", c_i64), ("C16", c_p),
        ("pre16", c_p), ("aux16", c_p), ("colsum_part", c_p), ("C16b", c_p),
    ]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64), ("nz1", c_i32), ("nz2", c_i32),
        ("A", Operand), ("B", Operand), ("ep", Epilogue),
        ("precision", c_i32), ("timing_family", c_i32), ("flops", c_f64),
        ("ksplit", c_i32), ("kchunk", c_i32), ("workspace", c_p), ("workspace_floats", c_i64),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "b2p_last_error": (ctypes.c_char_p, []),
    "b2p_version": (c_i32, []),
    "b2p_abi_sizes": (c_i32, [c_p]),
    "b2p_timing_enable": (c_i32, [c_i32, c_i32]),
    "b2p_timing_read": (c_i32, [c_i32, ctypes.POINTER(c_f32), ctypes.POINTER(c_i32), ctypes.POINTER(c_f64)]),
    "b2p_gemm": (c_i32, [ctypes.POINTER(GemmDesc), c_p]),
    "b2p_colsum_workspace": (c_i64, [c_i64, c_i64]),
    "b2p_colsum": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i32, c_p, c_p]),
    "b2p_colsum_batched": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_i32, c_p, c_p]),
    "b2p_colsum_parts": (c_i32, [c_p, c_i64, c_i64, c_p, c_i32, c_p]),
    "b2p_gemm16_variant": (c_i32, [c_i32]),
    "b2p_attn16_dkv_variant": (c_i32, [c_i32]),
    "b2p_set_gate_batch": (c_i32, [c_p]),
    "b2p_split3_bf16": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i32, c_i32, c_p]),
    "b2p_i64_fill": (c_i32, [c_p, ctypes.POINTER(c_i64), c_i32, c_p]),
    "b2p_colsum_pin_begin": (c_i32, []),
    "b2p_colsum_pin_end": (c_i64, []),
    "b2p_colsum_unpin": (c_i32, [c_i64]),
    "b2p_colsum_pool_state": (c_i64, [c_i64, ctypes.POINTER(c_i64)]),
    "b2p_dropout": (c_i32, [c_p, c_p, c_i64, c_f32, c_u64, c_p]),
    "b2p_layernorm_fwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, c_u64, c_p]),
    "b2p_layernorm_bwd_workspace": (c_i64, [c_i64, c_i64]),
    "b2p_layernorm_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_f32, c_u64,
                                  c_p, c_f32, c_u64, c_p, c_p, c_p]),
    "b2p_layernorm_fwd16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, c_u64, c_p]),
    "b2p_layernorm_bwd16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_f32, c_u64,
                                    c_p, c_f32, c_u64, c_p, c_p, c_p, c_p]),
    "b2p_layernorm_bwd_acc2": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_f32, c_u64,
                                       c_p, c_f32, c_u64, c_p, c_p, c_p, c_p]),
    "b2p_cast_bf16": (c_i32, [c_p, c_p, c_i64, c_p]),
    "b2p_softmax_fwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f32, c_u64, c_p]),
    "b2p_softmax_bwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f32, c_u64, c_p]),
    "b2p_act_bwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i32, c_p]),
    "b2p_gauss_smooth": (c_i32, [c_p, c_p, c_i32, c_p, c_i64, c_i64, c_i64, c_p]),
    "b2p_unfold_col2im": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_p]),
    "b2p_day_reduce": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p]),
    "b2p_unfold16": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_unfold_weight16": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_p, c_p]),
    "b2p_pad_rows16": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_cast16_tail": (c_i32, [c_p, c_p, c_i64, c_i64, c_i32, c_p]),
    "b2p_gather_recs": (c_i32, [c_p, c_i32, c_p]),
    "b2p_conv_weight_permute": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_conv_weight_transpose_flip": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_weight_norm_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "b2p_weight_norm_fwd": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p]),
    "b2p_weight_norm_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p]),
    "b2p_gru_fwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_gru_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_gru16_supported": (c_i32, [c_i64]),
    "b2p_gru16_lane_floats": (c_i64, [c_i64, c_i64, c_i64, c_i32, c_i32]),
    "b2p_gru_lane_permute": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_u32, c_i32, c_p]),
    "b2p_gru_fwd16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_gru_bwd16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_gru_mc_supported": (c_i32, [c_i64]),
    "b2p_gru_mc_workspace": (c_i64, [c_i64, c_i64, c_i32]),
    "b2p_gru_fwd_mc": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_gru_bwd_mc": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_gru_mc_status": (c_i32, [c_p, c_p, c_i32, c_p]),
    "b2p_gru_mc_debug_withhold": (c_i32, [c_i32]),
    "b2p_gru_hprev": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_attn16_fwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_u64, c_p, c_p]),
    "b2p_attn16_fwd_f16": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_u64, c_p, c_p]),
    "b2p_attn16_fwd_keep": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_p, c_p]),
    "b2p_attn16_fwd_f16_keep": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_p, c_p]),
    "b2p_attn16_keep_masks": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_p]),
    "b2p_attn16_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_u64, c_p,
                               c_p]),
    "b2p_attn16_bwd_f16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_f32, c_f32, c_u64, c_p,
                               c_p]),
    "b2p_ctc_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "b2p_ctc_fwd_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "b2p_adam_multi": (c_i32, [c_p, c_i32, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_p]),
    "b2p_adam_multi_dev": (c_i32, [c_p, c_i32, c_i64, c_p, c_f32, c_f32, c_f32, c_f32, c_p, c_p, c_p]),
    "b2p_cast16_2d": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i32, c_p]),
    "b2p_accum_recs": (c_i32, [c_p, c_i32, c_p]),
    "b2p_accum_rows_recs": (c_i32, [c_p, c_i32, c_p]),
    "b2p_adam_recs": (c_i32, [c_p, c_i32, c_f32, c_f64, c_f64, c_f32, c_f32, c_f32, c_f32, c_p, c_p, c_p, c_p]),
    "b2p_adam_gated_recs": (c_i32, [c_p, c_i32, c_p, c_f64, c_f64, c_f32, c_f32, c_p, c_p]),
    "b2p_set_seed_epoch": (c_i32, [c_p]),
    "b2p_ctc_greedy_wer": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "b2p_ctc_beam_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "b2p_ctc_prefix_beam": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i32, c_f32, c_f32, c_p, c_p, c_p, c_p, c_p]),
    "b2p_ctc_greedy_cer": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "b2p_transpose_bf16": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_posconv16_fwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_posconv16_bwd_data": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_posconv16_wgrad": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_seed_epoch_step": (c_i32, [c_p, c_p]),
    "b2p_scale_by_device_scalar": (c_i32, [c_p, c_p, c_p, c_i64, c_p]),
    "b2p_unfold_lens": (c_i32, [c_p, c_p, c_i64, c_i64, c_i64, c_p]),
    "b2p_ctc_targets": (c_i32, [c_p, c_p, c_i64, c_p]),
    "b2p_dropout_scaled": (c_i32, [c_p, c_p, c_i64, c_f32, c_u64, c_f32, c_p]),
    "b2p_drop_cast_colsum_parts": (c_i64, [c_i64]),
    "b2p_drop_cast_colsum": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_f32, c_u64, c_f32, c_p]),
    "b2p_layernorm_fwd_x16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_p]),
    "b2p_glu_bwd16": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_p]),
    "b2p_rotary16": (c_i32, [c_p, c_p, c_p, c_p, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_p]),
    "b2p_layernorm_rotary16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_i64, c_i64, c_p, c_p, c_i32,
                                       c_p, c_p, c_p, c_p, c_p]),
    "b2p_act_dropout_cast16": (c_i32, [c_p, c_p, c_i64, c_i32, c_f32, c_u64, c_p]),
    "b2p_rotary": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_glu_fwd": (c_i32, [c_p, c_p, c_i64, c_i64, c_p]),
    "b2p_glu_bwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_p]),
    "b2p_dwconv_fwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p]),
    "b2p_dwconv_bwd_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i32]),
    "b2p_dwconv_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p, c_p]),
    "b2p_batchnorm_workspace": (c_i64, [c_i64, c_i64]),
    "b2p_batchnorm_fwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, c_i32,
                                  c_p, c_p]),
    "b2p_batchnorm_eval": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_i32, c_p, c_p]),
    "b2p_batchnorm_bwd": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i32, c_p, c_p]),
    "b2p_batchnorm_stats": (c_i32, [c_p, c_p, c_p, c_i64, c_i64, c_p, c_p]),
    "b2p_batchnorm_count_next": (c_i32, [c_p]),
    "b2p_batchnorm_fwd16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32,
                                    c_f32, c_i32, c_p, c_p]),
    "b2p_batchnorm_apply16": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_i64, c_i64, c_i32, c_p]),
    "b2p_batchnorm_finalize": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f32, c_f32, c_i32, c_p]),
    "b2p_batchnorm_apply": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i32, c_p]),
    "b2p_batchnorm_bwd_sums": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i32, c_p, c_p]),
    "b2p_batchnorm_bwd_dx": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p]),
    "b2p_layerdrop_keep": (c_i32, [c_f32, c_u64, c_u64, c_i32, ctypes.POINTER(c_i32)]),
    "b2p_layerdrop_select": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_f32, c_u64, c_p]),
    "b2p_layerdrop_select_h": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_f32, c_u64, c_p]),
    "b2p_layerdrop_route": (c_i32, [c_p, c_p, c_p, c_i64, c_f32, c_u64, c_p]),
    "b2p_set_gate": (c_i32, [c_p]),
    "b2p_layerdrop_flag": (c_i32, [c_p, c_f32, c_u64, c_p]),
}

# timing families (b2p_timing_*)
TIMING_GEMM = 1
EPI_C16_FP16 = 1   # b2p_epilogue.flags: C16 holds fp16 bits (include/b2p_hip.h B2P_EPI_C16_FP16)

_lib = None


def load() -> ctypes.CDLL:
    """Loads the HIP library (raises if absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: build it with `python -m wav2vec2forbrain_amd.build_lib` "
            "(or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return list(_SIGS)


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().b2p_last_error().decode(errors="replace")
        raise RuntimeError(f"b2p HIP library error in {what}: {msg} (rc={rc})")


def call(name: str, *args) -> None:
    """Calls a status-returning entry point and raises RuntimeError on failure."""
    rc = getattr(load(), name)(*args)
    check(rc, name)


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()
