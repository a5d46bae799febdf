"""ctypes binding of libospo_hip.so (the C ABI declared in include/ospo_hip.h).

The product path has NO fallback: if the library is missing or a call returns
a non-zero ospo_status, this raises.  ``ValueError`` for shape/argument
violations (mirroring ``ospo/wrapper/train.py:382-383,335-337``), ``RuntimeError``
for HIP launch failures.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_long, c_size_t, c_uint, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OSPO_HIP_LIB", os.path.join(_HERE, "libospo_hip.so"))

P, I, L, F, Z, U = c_void_p, c_int, c_long, c_float, c_size_t, c_uint

# include/ospo_hip.h OSPO_ABI_VERSION: a library built from other sources (another workspace layout, other
# dropout masks) is refused at load instead of silently mis-driven
ABI_VERSION = 3

# name -> argtypes (restype is c_int = ospo_status unless listed in RESTYPES)
SIGNATURES = {
    "ospo_abi_version": [],
    "ospo_ws_counter_bytes": [I],
    "ospo_gemm_clock_probe_bf16": [P, P, P, I, I, I, P, Z, P],
    "ospo_dropout_hash": [U, U],
    "ospo_gemm_nt_bf16": [P, I, P, I, I, I, I, P, I, P, I, I, F, P, P, I, P, I, I, P, Z, P],
    "ospo_gemm_nt_ws_bytes": [I, I, I, I, I, I],
    "ospo_gemm_nt_tile": [I, I],
    "ospo_gemm_nt_dropout_bf16": [P, I, P, I, I, I, I, P, I, P, I, I, P, I, U, F, P, I, P, Z, P],
    "ospo_gemm_nt_swiglu_bwd_bf16": [P, I, P, I, I, I, I, P, I, P, I, I, P, I, P, I, U, F, I, P, Z, P],
    "ospo_gemm_nt_rope_bf16": [P, I, P, I, I, I, I, P, I, P, I, I, P, I, P, P, I, I, I, P, Z, P],
    "ospo_mx8_scale_bytes": [I, I],
    "ospo_quant_mx8": [P, I, I, I, P, I, P, P],
    "ospo_gemm_nt_mx8": [P, I, P, P, I, P, I, I, I, P, I, P, I, I, F, P, P, I, P, I, P, P, I, I, U, F, I, P, Z, P],
    "ospo_gemm_f32acc": [P, I, I, P, I, I, I, I, I, I, F, P, I, I, I, P],
    "ospo_gemm_f32acc_bdrop": [P, I, I, P, I, I, I, I, I, I, F, P, I, I, I, U, F, P, P],
    "ospo_lora_wgrad": [P, I, I, P, I, I, I, I, I, I, P, I, I, U, F, P],
    "ospo_lora_da": [P, I, I, P, I, I, I, P, I, I, U, F, P, P],
    "ospo_swiglu_fwd_lora_down": [P, I, P, I, I, I, I, P, I, I, I, F, P, I, I, P, Z, U, F, P, P],
    "ospo_f32_to_bf16": [P, P, L, F, P],
    "ospo_rmsnorm_fwd": [P, P, P, P, I, I, F, P],
    "ospo_rmsnorm_bwd": [P, P, P, P, P, P, I, I, P],
    "ospo_rope_fwd": [P, I, I, I, I, I, I, I, P, P, P],
    "ospo_rope_bwd": [P, I, I, I, I, I, I, I, P, P, P],
    "ospo_swiglu_fwd": [P, I, P, I, I, I, P],
    "ospo_rmsnorm_fwd_mx8": [P, P, P, P, I, I, F, P, I, P, P],
    "ospo_rmsnorm_bwd_mx8": [P, P, P, P, P, P, I, I, P, I, P, P],
    "ospo_swiglu_fwd_mx8": [P, I, P, I, I, I, P, I, P, P],
    "ospo_swiglu_bwd_mx8": [P, I, P, I, P, I, I, I, P, I, P, P],
    "ospo_swiglu_bwd": [P, I, P, I, P, I, I, I, P],
    "ospo_flash_attn_fwd": [P, I, I, I, I, P, I, P, I, I, I, I, F, P],
    "ospo_flash_attn_bwd": [P, I, I, I, I, P, I, P, I, P, P, P, P, I, I, I, I, I, F, P, P, P],
    "ospo_flash_attn_bwd_ws_bytes": [I, I, I],
    "ospo_flash_attn_fwd_mx8": [P, I, I, I, I, P, I, P, I, I, I, I, F, P, I, P, I, P],
    "ospo_flash_attn_bwd_mx8": [P, I, I, I, I, P, I, P, I, P, P, P, P, I, I, I, I, I, F, P, P, P, I, P, I, P],
    "ospo_assemble_inputs": [P, I, I, P, I, P, I, I, P, P],
    "ospo_gen_aligner_in": [P, I, P, I, I, P, P, I, P, P],
    "ospo_gather_rows": [P, I, I, I, I, I, I, P, P],
    "ospo_scatter_rows": [P, I, I, I, I, I, P, I, I, P],
    "ospo_row_dot_sum": [P, L, I, I, I, P, P, F, I, P, P, Z, P],
    "ospo_row_dot_sum_ws_bytes": [I, I, I],
    "ospo_gelu_fwd": [P, P, L, P],
    "ospo_gelu_bwd": [P, P, P, L, P],
    "ospo_logprob_fwd": [P, I, P, I, I, P, P, P, P],
    "ospo_logprob_bwd": [P, I, P, P, I, I, P, P, P],
    "ospo_simpo_fwd": [P, I, F, F, F, I, P, P, P, P],
    "ospo_simpo_bwd": [P, I, F, F, F, I, P, P, P],
    "ospo_lora_pack": [P, P, I, I, I, I, I, P, P, P, P, I, L, P],
    "ospo_lora_gdb": [P, I, P, I, P, I, I, I, I, I, F, P, I, I, P, P, Z, P],
    "ospo_lora_gdb_r": [P, I, P, I, P, I, I, I, I, I, I, F, P, I, I, P, P, Z, P],
    "ospo_lora_gdb_ws_bytes": [I, I, I],
    "ospo_swiglu_lora_gdb": [P, I, P, I, P, I, P, I, P, I, I, I, I, F, P, I, I, P, P, Z, P],
    "ospo_swiglu_lora_gdb_r": [P, I, P, I, P, I, P, I, P, I, I, I, I, I, F, P, I, I, P, P, Z, P],
    "ospo_lora_skinny": [P, I, P, I, I, I, I, I, I, I, I, F, P, I, I, P, Z, U, F, P, I, P, P],
    "ospo_lora_skinny_ws_bytes": [I, I, I],
    "ospo_decode_gemv_ws_bytes": [I, I, I],
    "ospo_decode_gemv_fusable": [I, I, I],
    "ospo_decode_gemv_kv": [P, I, P, I, I, I, I, I, P, Z, P, P, P, P, P, I, P, I, P],
    "ospo_decode_gemv_swiglu": [P, I, P, I, I, I, I, P, Z, P, I, P],
    "ospo_decode_gemv": [P, I, P, I, I, I, I, P, I, P, I, P, I, P, Z, P],
    "ospo_decode_linear_ws_bytes": [I, I, I],
    "ospo_decode_linear": [P, P, I, I, I, I, P, I, P, F, I, P, I, P, I, P, I, P, P, P, P, P, P, I, I, P, Z, P],
    "ospo_decode_mlp": [P, P, P, I, I, I, I, P, I, P, F, P, I, P, I, P, P, I, P, P, P, Z, P],
    "ospo_decode_attn_o": [P, I, P, P, I, I, I, P, P, F, P, I, P, P, I, P, I, P, P, I, P, P, P, Z, P],
    "ospo_decode_qkv_heads": [P, P, I, I, I, P, I, P, F, P, I, P, P, P, P, P, I, I, I, I, P, Z, P],
    "ospo_attn_cache_heads": [P, I, P, P, I, I, I, I, I, I, P, P, F, P, I, P],
    "ospo_kv_store": [P, I, I, I, P, I, P, P, P, P, I, I, I, P, I, P],
    "ospo_attn_cache": [P, I, P, P, I, I, I, I, I, P, P, F, P, I, P],
    "ospo_cfg_sample": [P, I, I, I, F, F, P, P, I, P, P, P, P],
    "ospo_embed_rows": [P, L, P, I, I, P, P],
    "ospo_decode_advance": [P, P, P],
    "ospo_vq_conv2d": [P, I, I, I, I, P, I, I, I, I, I, I, I, I, P, P, P, P],
    "ospo_vq_bmm_nt": [P, P, I, I, I, I, P, P],
    "ospo_vq_groupnorm_ws_bytes": [I, I],
    "ospo_vq_groupnorm": [P, I, I, I, I, P, P, F, I, P, P, Z, P],
    "ospo_vq_softmax_rows": [P, I, I, F, P],
    "ospo_vq_transpose": [P, I, I, I, P, P],
    "ospo_vq_l2norm_rows": [P, L, I, P, P],
    "ospo_vq_quantize": [P, L, I, P, I, P, P, P],
    "ospo_vq_embed_codes": [P, L, P, I, I, P, P],
    "ospo_vq_conv2d_up2": [P, I, I, I, I, P, I, I, I, I, P, P, P, P],
    "ospo_vq_to_uint8": [P, L, P, P],
    "ospo_sumsq": [P, L, P, P, P],
    "ospo_adamw_clip": [P, P, P, P, L, F, F, F, F, F, I, P, F, P],
}

# include/ospo_hip_ablation.h: only in libospo_hip_ablation.so (tools/ A/B runs, OSPO_HIP_LIB=...)
ABLATION_SIGNATURES = {"ospo_set_gemm_variant": [I], "ospo_set_gemv_variant": [I], "ospo_set_gemv_splits": [I],
                       "ospo_set_skinny_variant": [I], "ospo_gemm_set_debug_buffer": [P],
                       "ospo_attn_set_stamps": [P]}

RESTYPES = {"ospo_ws_counter_bytes": c_size_t, "ospo_gemm_nt_ws_bytes": c_size_t, "ospo_row_dot_sum_ws_bytes": c_size_t, "ospo_lora_gdb_ws_bytes": c_size_t, "ospo_flash_attn_bwd_ws_bytes": c_size_t, "ospo_lora_skinny_ws_bytes": c_size_t, "ospo_mx8_scale_bytes": c_size_t, "ospo_decode_gemv_ws_bytes": c_size_t, "ospo_decode_linear_ws_bytes": c_size_t, "ospo_vq_groupnorm_ws_bytes": c_size_t, "ospo_dropout_hash": c_uint}

_lib = None


class OspoError(RuntimeError):
    pass


def lib():
    """Load the library once; raise loudly when it is absent (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OspoError(f"libospo_hip.so not found at {LIB_PATH}: build it with "
                            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        h = ctypes.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = argt
            fn.restype = RESTYPES.get(name, c_int)
        for name, argt in ABLATION_SIGNATURES.items():
            if hasattr(h, name):
                fn = getattr(h, name)
                fn.argtypes = argt
                fn.restype = c_int
        h.ospo_strerror.argtypes = [c_int]
        h.ospo_strerror.restype = ctypes.c_char_p
        if h.ospo_abi_version() != ABI_VERSION:
            raise OspoError(f"{LIB_PATH}: ABI version {h.ospo_abi_version()}, this binding needs {ABI_VERSION} "
                            "(rebuild the library from this tree)")
        _lib = h
    return _lib


def exported_symbols():
    return list(SIGNATURES) + ["ospo_strerror"]


def query(name: str, *args) -> int:
    """Call an entry point that returns a value rather than a status."""
    return getattr(lib(), name)(*args)


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().ospo_strerror(rc).decode()
        if rc in (1, 2, 5):
            raise ValueError(f"{name}: {msg} (status {rc})")
        raise OspoError(f"{name}: {msg} (status {rc})")
