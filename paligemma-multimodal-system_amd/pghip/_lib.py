"""ctypes binding of libpghip.so (the C-ABI declared in include/pghip.h).

There is no fallback: if the library is missing or a call fails, this raises.
Import torch before loading so the HIP runtime torch ships is the one the library
binds to (same soname, libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PGHIP_LIB selects a tuning build of the same sources (scripts/tune/); default: the in-tree product build
LIB_PATH = os.environ.get("PGHIP_LIB") or os.path.join(_HERE, "libpghip.so")

vp, i32, i64, f32, u32 = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_uint

class PgFusedArgs(C.Structure):
    """Mirror of PgFusedArgs (include/pghip.h)."""
    _fields_ = [("pro_mode", C.c_int), ("resid_in", C.c_void_p), ("resid_out", C.c_void_p),
                ("partials", C.c_void_p), ("nsplit", C.c_int), ("norm_w", C.c_void_p), ("eps", C.c_float),
                ("part_o", C.c_void_p), ("part_ml", C.c_void_p), ("asplit", C.c_int), ("head_dim", C.c_int),
                ("dtw", C.c_int), ("q_per_kv", C.c_int), ("kv_heads", C.c_int), ("cos_t", C.c_void_p),
                ("sin_t", C.c_void_p), ("pos", C.c_void_p), ("rows_per_batch", C.c_int), ("slot_dev", C.c_void_p),
                ("slot_base", C.c_int), ("kc", C.c_void_p), ("vtc", C.c_void_p), ("smax", C.c_int),
                ("q_heads", C.c_int), ("fin_cnt", C.c_void_p), ("fin_resid", C.c_void_p), ("ss_out", C.c_void_p),
                ("ss_in", C.c_void_p), ("ss_ld", C.c_int), ("ss_n", C.c_int), ("fin_x", C.c_void_p),
                ("akeys", C.c_int), ("a_scale", C.c_void_p), ("w_scale", C.c_void_p),
                ("slab_rows", C.c_int), ("kd", C.c_void_p), ("vd", C.c_void_p),
                ("amax_out", C.c_void_p), ("amax_in", C.c_void_p), ("amax_ld", C.c_int), ("amax_zero", C.c_void_p),
                ("amax_zero_n", C.c_int), ("fx", C.c_void_p),
                ("mx_out", C.c_void_p), ("mx_in", C.c_void_p), ("status", C.c_void_p)]


# name -> argtypes (every function returns int: 0 or a hipError_t code)
SIGNATURES = {
    "pg_abi_version": [],
    "pg_source_hash": [C.c_char_p, i32],
    "pg_gemm": [vp, i32, vp, i32, vp, vp, i32, i32, i32, i32, i32, i32, vp, i32, vp, i32, i32, vp],
    "pg_gemm_fused": [vp, i32, vp, i32, vp, vp, i32, i32, i32, i32, i32, i32, C.POINTER(PgFusedArgs), vp],
    "pg_gemm_finalize": [vp, i32, vp, i32, i32, i32, i32, vp, i32, i32, C.POINTER(PgFusedArgs), vp],
    "pg_norm_residual": [vp, vp, i32, i32, vp, vp, vp, i32, vp, vp, i32, i32, i32, f32, i32, vp],
    "pg_attention": [vp, i64, vp, i64, vp, i64, i64, i64, vp, i64, i64, i64, vp, i64, i64,
                     i32, i32, i32, vp, i32, i32, i32, f32, i32, i32, vp, vp, i32, vp, vp, vp],
    "pg_attn_combine": [vp, vp, i32, i32, i32, i32, i32, vp, i64, vp],
    "pg_attn_probs": [vp, i64, vp, i64, i64, i64, vp, i64, i64, i32, i32, i32, i32, i32, i32, f32, i32, vp, vp],
    "pg_attn_decode": [vp, i64, vp, i64, vp, vp, i32, i32, vp, i32, i32, i32, f32, i32, i32, i32, i32, vp, vp, vp,
                       vp, vp, i64, vp],
    "pg_rope_kv_write": [vp, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, i32, vp, vp],
    "pg_patch_im2col": [vp, i32, i32, i32, i32, i32, vp, i32, vp],
    "pg_image_rank": [vp, i32, i64, vp, vp],
    "pg_embed_merge": [vp, vp, i32, vp, i32, vp, i32, i32, i64, i64, f32, f32, vp, vp],
    "pg_argmax": [vp, i64, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp],
    "pg_argmax_embed": [vp, i64, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, i32, vp, i32, i32, i64, i64, f32, f32, vp,
                        vp],
    "pg_argmax_pairs": [vp, i64, i32, i32, i32, vp, vp, vp],
    "pg_argmax_merge": [vp, i32, i32, vp, vp, i32, vp, vp, vp, vp],
    "pg_topp_sample": [vp, i64, i32, i32, f32, f32, vp, vp, vp, i32, vp, vp, vp, vp, vp],
    "pg_image_preprocess": [vp, i32, i32, i32, vp, vp, i32, vp, vp, i32, i32, i32, vp, vp, vp, vp],
    "pg_synth_fill": [vp, i64, u32, f32, f32, i32, vp],
    "pg_quant_fp8": [vp, i32, i32, i32, vp, i32, vp, vp],
    "pg_norm_residual_fp8": [vp, vp, i32, i32, vp, vp, vp, i32, vp, vp, i32, i32, i32, f32, i32, vp],
    "pg_norm_residual_mx": [vp, vp, i32, i32, vp, vp, i32, vp, vp, i32, i32, i32, i32, vp],
    "pg_xgmi_buffer_bytes": [i32, i64, C.POINTER(C.c_long)],
    "pg_xgmi_alloc": [i64, C.POINTER(C.c_void_p)],
    "pg_xgmi_free": [vp],
    "pg_xgmi_ipc_handle": [vp, C.c_char_p],
    "pg_xgmi_ipc_open": [C.c_char_p, C.POINTER(C.c_void_p)],
    "pg_xgmi_ipc_close": [vp],
    "pg_allreduce_xgmi": [vp, i64, i32, i32, C.POINTER(C.c_void_p), i64, vp, vp, vp],
    "pg_allreduce_xgmi_slabs": [vp, i64, i32, i64, i32, i32, C.POINTER(C.c_void_p), i64, vp, vp, vp],
    "pg_allgather_xgmi": [vp, i64, vp, i32, i32, C.POINTER(C.c_void_p), i64, vp, vp, vp],
    "pg_xgmi_rs_buffer_bytes": [i32, i64, C.POINTER(C.c_long)],
    "pg_allreduce_xgmi_rs": [vp, i64, i32, i64, i32, i32, C.POINTER(C.c_void_p), i64, i32, vp, vp, vp],
}

_lib = None
_hip = None


class PgHipError(RuntimeError):
    pass


ABI_VERSION = 13


def source_hash(lib=None) -> str:
    """The source hash compiled into the loaded library (pg_source_hash)."""
    lib = load() if lib is None else lib
    buf = C.create_string_buffer(80)
    if lib.pg_source_hash(buf, 80) != 0:
        raise PgHipError("pg_source_hash: buffer too small")
    return buf.value.decode()


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libpghip.so.  The product library must match this tree: its ABI version and the source hash compiled
    into it (pghip/build.py) are checked against include/pghip.h's ABI and the csrc/ sources next to it, so a stale
    prebuilt library raises instead of running (PGHIP_LIB, a tuning build, skips the source check)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise PgHipError(f"libpghip.so not found at {path}: build it with `python -m pghip.build` "
                         "(or __graft_entry__.build()); there is no CPU fallback.")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = C.c_int
    if lib.pg_abi_version() != ABI_VERSION:
        raise PgHipError(f"{path}: ABI {lib.pg_abi_version()}, this package expects {ABI_VERSION}; rebuild it")
    if not os.environ.get("PGHIP_LIB"):
        from . import build
        if os.path.isdir(build.CSRC):
            want, got = build.source_hash(), source_hash(lib)
            if want != got:
                raise PgHipError(f"{path} was built from other sources (hash {got[:16]}, tree {want[:16]}): "
                                 "rebuild it with `python -m pghip.build`")
    _lib = lib
    return lib


def _err_string(code: int) -> str:
    global _hip
    try:
        if _hip is None:
            _hip = C.CDLL("libamdhip64.so.7")
            _hip.hipGetErrorString.restype = C.c_char_p
            _hip.hipGetErrorString.argtypes = [C.c_int]
        return _hip.hipGetErrorString(code).decode()
    except Exception:  # pragma: no cover
        return "?"


def call(name: str, *args) -> None:
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise PgHipError(f"{name} failed: hip error {rc} ({_err_string(rc)})")
