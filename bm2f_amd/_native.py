"""ctypes binding of ``libbm2f.so`` (the C ABI declared in ``include/bm2f.h``).

The library is built in-tree (``bm2f_amd/lib/libbm2f.so``, see ``bm2f_amd/build.py``) so it travels
with the repository snapshot to the GPU box.  There is no fallback: if the library is missing or
fails to load, every op raises.  This mirrors the reference's hard dependency on its compiled
``MultiScaleDeformableAttention`` module (ops/functions/ms_deform_attn_func.py:21-29), minus the
reference's silent pure-PyTorch fallback (ops/modules/ms_deform_attn.py:116-121).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libbm2f.so")
_lock = threading.Lock()
_lib = None

ABI_VERSION = 1

_p = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_l = ctypes.c_int64

# name -> argtypes (all return int status)
_SIGNATURES = {
    "m2f_msda_fwd_f32": [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p],
    "m2f_msda_fwd_f64": [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p],
    "m2f_msda_bwd_f32": [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p],
    "m2f_msda_bwd_f64": [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p],
    "m2f_msda_fused_fwd_f32": [_p, _p, _i, _p, _l, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p],
    "m2f_msda_fused_bwd_workspace": [_p, _i, _i, _i, _i, _i, _i, _p],
    "m2f_msda_fused_bwd_f32": [_p, _p, _i, _p, _l, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _l, _p],
    "m2f_msda_fused_fwd_hm_f32": [_p, _p, _i, _p, _l, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p],
    "m2f_msda_fused_bwd_hm_f32": [_p, _p, _i, _p, _l, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _l, _p],
    "m2f_attn_mask_bits": [_p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _i, _p],
    "m2f_mask_heads_fwd": [_i, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _i, _p],
    "m2f_mask_row_fix": [_p, _i, _i, _i, _p],
    "m2f_mask_heads_bwd_workspace": [_i, _i, _l, _p],
    "m2f_mask_heads_bwd_embed": [_i, _p, _p, _i, _i, _i, _l, _p, _p, _l, _p],
    "m2f_mask_heads_bwd_feats": [_i, _p, _i, _p, _i, _i, _i, _i, _l, _i, _p, _p],
    "m2f_masked_attn_plan": [_i, _i, _i, _i, _p, _p, _p, _p],
    "m2f_masked_attn_fwd": [_i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _f, _p, _p, _p, _l, _p],
    "m2f_masked_attn_bwd": [_i, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _f, _p, _p, _p, _p,
                            _l, _p],
    "m2f_gemm_f32_nt": [_p, _l, _p, _l, _p, _i, _p, _l, _p, _l, _i, _i, _i, _p],
    "m2f_gemm_f32_tn_workspace": [_i, _i, _i, _p],
    "m2f_gemm_f32_tn": [_p, _l, _p, _l, _p, _l, _p, _i, _i, _i, _p, _l, _p],
    "m2f_gemm_f32x3_nt_workspace": [_i, _i, _p],
    "m2f_gemm_f32x3_nt": [_p, _l, _p, _l, _i, _p, _i, _p, _l, _p, _l, _i, _i, _i, _p, _l, _p],
    "m2f_gemm_f32x3_nt_add": [_p, _l, _p, _l, _i, _p, _i, _p, _l, _p, _p, _l, _p, _l, _i, _i, _i, _p, _l, _p],
    "m2f_gemm_f32x3_nt_bits": [_p, _l, _p, _l, _i, _p, _i, _p, _p, _l, _p, _l, _i, _i, _i, _p, _l, _p],
    "m2f_gemm_f32x3_nt_rowadd": [_p, _l, _p, _l, _i, _p, _l, _i, _p, _l, _i, _i, _i, _p, _l, _p],
    "m2f_gemm_f32x3_tn_workspace": [_i, _i, _i, _p],
    "m2f_gemm_f32x3_tn": [_p, _l, _p, _l, _p, _l, _p, _i, _i, _i, _p, _l, _p],
    "m2f_conv_f32x3_workspace": [_i, _i, _i, _i, _i, _i, _p],
    "m2f_conv_f32x3": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p, _l, _p],
    "m2f_conv_f32x3_wgrad": [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _l, _p],
    "m2f_conv_x3_io": [_p, _i, _i, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _l, _p],
    "m2f_conv_x3_wgrad_io": [_p, _p, _i, _i, _p, _p, _i, _i, _i, _i, _i, _i, _p, _l, _p],
    "m2f_bias_act_nchw": [_p, _p, _p, _l, _i, _l, _i, _i, _p],
    "m2f_relu_bwd_sum": [_p, _i, _p, _p, _l, _i, _p],
    "m2f_upsample2x_add_fwd_f32": [_p, _l, _l, _l, _l, _p, _p, _i, _i, _i, _i, _p],
    "m2f_upsample2x_bwd_f32": [_p, _p, _i, _i, _i, _i, _p],
    "m2f_upsample2x_add_fwd_nhwc_f32": [_p, _l, _p, _p, _i, _i, _i, _i, _p],
    "m2f_upsample2x_bwd_nhwc_f32": [_p, _p, _i, _i, _i, _i, _p],
    "m2f_maxpool3s2_fwd": [_p, _p, _p, _l, _i, _i, _i, _p],
    "m2f_maxpool3s2_bwd": [_p, _p, _p, _l, _i, _i, _i, _p],
    "m2f_maxpool3s2_nhwc": [_i, _p, _p, _p, _i, _i, _i, _i, _i, _p],
    "m2f_stream_copy": [_p, _p, _l, _i, _p],
    "m2f_gather_probe": [_p, _i, _l, _p, _i, _p],
    "m2f_set_option": [ctypes.c_char_p, _l],
    "m2f_get_option": [ctypes.c_char_p, _p],
    "m2f_transpose_f32": [_p, _l, _l, _p, _l, _l, _i, _i, _i, _p],
    "m2f_colsum_workspace": [_l, _i, _p],
    "m2f_colsum": [_i, _p, _l, _i, _p, _l, _p, _p],
    "m2f_sum_to_f32": [_p, _i, _l, _i, _p, _p],
    "m2f_group_norm_workspace": [_i, _i, _i, _l, _p],
    "m2f_group_norm_fwd_f32": [_p, _p, _p, _i, _i, _i, _l, _f, _i, _p, _p, _p, _p, _l, _p],
    "m2f_group_norm_bwd_f32": [_p, _p, _p, _p, _p, _p, _i, _i, _i, _l, _i, _p, _p, _p, _p, _l, _p],
    "m2f_add_layernorm_workspace": [_l, _i, _p],
    "m2f_add_layernorm_fwd_f32": [_p, _p, _p, _p, _l, _i, _f, _p, _p, _p, _p],
    "m2f_add_layernorm_bwd_f32": [_p, _p, _p, _p, _p, _p, _l, _i, _p, _p, _p, _p, _l, _p],
    "m2f_lsap_batched": [_p, _i, _i, _i, _l, _p, _p, _p, _p, _p],
    "m2f_pairwise_tiles": [_i, _i],
    "m2f_pairwise_rows": [_p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _p],
    "m2f_pairwise_match_cost": [_p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _p, _p],
    "m2f_pairwise_rows_bwd": [_p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p],
    "m2f_threshold_bits": [_p, _i, _l, _f, _p, _p],
    "m2f_weaksup_lab": [_p, _i, _i, _i, _i, _p, _p],
    "m2f_color_similarity": [_p, _p, _i, _i, _i, _i, _p, _p],
}


class NativeError(RuntimeError):
    """A nonzero status returned by libbm2f (message from ``m2f_last_error``)."""


def library_path() -> str:
    return _LIB_PATH


def load():
    """Load (once) and return the ctypes handle; raises ImportError when the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise ImportError(
                f"libbm2f.so not found at {_LIB_PATH}; build it with `python -c \"import __graft_entry__ as g; g.build()\"` "
                "or `python -m bm2f_amd.build`")
        lib = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        lib.m2f_last_error.restype = ctypes.c_char_p
        lib.m2f_last_error.argtypes = []
        lib.m2f_abi_version.restype = ctypes.c_int
        lib.m2f_abi_version.argtypes = []
        got = lib.m2f_abi_version()
        if got != ABI_VERSION:
            raise ImportError(f"libbm2f.so ABI version {got} != expected {ABI_VERSION}; rebuild it")
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _lib = lib
        return lib


def exported_symbols():
    return ["m2f_last_error", "m2f_abi_version", *_SIGNATURES.keys()]


def call(name: str, *args) -> None:
    """Invoke ``name`` and raise NativeError (a RuntimeError) on a nonzero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.m2f_last_error().decode("utf-8", "replace")
        raise NativeError(f"{name} failed (code {rc}): {msg}")


def set_option(name: str, value: int) -> None:
    """m2f_set_option: a geometry / engine override (value < 0 restores the default)."""
    call("m2f_set_option", name.encode(), int(value))


def get_option(name: str) -> int:
    v = ctypes.c_int64()
    call("m2f_get_option", name.encode(), ctypes.byref(v))
    return v.value


@contextlib.contextmanager
def options(**kw):
    """Set native options for the duration of a with-block (tests sweep geometries this way)."""
    old = {k: get_option(k) for k in kw}
    try:
        for k, v in kw.items():
            set_option(k, v)
        yield
    finally:
        for k, v in old.items():
            set_option(k, v)
