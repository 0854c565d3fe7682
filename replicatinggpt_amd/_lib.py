"""ctypes binding of libcharpt_hip.so (the C ABI declared in include/charpt.h).

The library is built in-tree (``python __graft_entry__.py`` / ``make -C replicatinggpt_amd/csrc``)
and must be present: there is no CPU or eager-PyTorch fallback for the product path.
"""
import ctypes
import os
import re

import torch  # noqa: F401  -- load torch's HIP runtime first so the library binds to the same one

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CHARPT_LIB") or os.path.join(_HERE, "libcharpt_hip.so")   # CHARPT_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "charpt.h")

CG_F32, CG_BF16, CG_BITS = 0, 1, 2
EPI_STORE, EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_RESID, EPI_BIAS_DROP_RESID, EPI_RELU_BWD = range(6)
EPI_STORE_ROWDOT = 7
GEMM_SLAB_BF16, GEMM_DEFER_REDUCE = 1, 2   # cg_epilogue_t.flags (per call: precision / deferral)
DEFER = 1                                  # flags of the _ex column-sum reduces

c_i64, c_int, c_dbl, c_flt, c_u64, P = ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p


class Epilogue(ctypes.Structure):
    _fields_ = [("kind", c_int), ("bias", P), ("resid", P), ("ld_resid", c_i64), ("aux", P), ("aux_dtype", c_int),
                ("ld_aux", c_i64), ("dropout_p", c_dbl), ("seed", c_u64), ("rng_call", P), ("site", c_int),
                ("beta", c_flt), ("colpart", P), ("flags", c_int)]


_SIGS = {
    "cg_last_error_string": (ctypes.c_char_p, []),
    "cg_version": (c_int, []),
    "cg_set_tuning": (c_int, [ctypes.c_char_p, c_int]),
    "cg_device_info": (c_int, [P, P, P]),
    "cg_counter_add": (c_int, [P, c_i64, P]),
    "cg_rng_snapshot": (c_int, [P, P, P]),
    "cg_dropout_mask": (c_int, [P, c_i64, c_dbl, c_u64, P, c_int, P]),
    "cg_dropout_apply": (c_int, [P, c_i64, c_i64, c_i64, P, c_int, c_dbl, c_u64, P, c_int, P]),
    "cg_sum_f32": (c_int, [P, c_i64, c_flt, P, P, P]),
    "cg_cast_f32_bf16": (c_int, [P, P, c_i64, P]),
    "cg_gather_batch": (c_int, [P, c_int, P, P, P, c_i64, c_i64, P]),
    "cg_embed_fwd": (c_int, [P, P, P, P, c_i64, c_i64, c_i64, c_i64, P]),
    "cg_embed_bwd_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "cg_embed_bwd": (c_int, [P, P, P, P, c_i64, c_i64, c_i64, c_i64, c_int, P, P]),
    "cg_layernorm_fwd": (c_int, [P, P, P, P, c_int, P, P, c_i64, c_i64, c_flt, P]),
    "cg_layernorm_bwd_workspace": (c_i64, [c_i64, c_i64]),
    "cg_layernorm_bwd": (c_int, [P, c_int, P, P, P, P, P, P, P, P, P, c_int, P, c_i64, c_i64, P]),
    "cg_layernorm_bwd_ex": (c_int, [P, c_int, P, P, P, P, P, P, P, c_dbl, c_u64, P, c_int, P, P, P, c_int, c_int, P,
                                    c_i64, c_i64, P]),
    "cg_layernorm_bwd_rows": (c_int, [P, c_int, P, P, P, P, P, P, P, c_dbl, c_u64, P, c_int, c_int, P, c_i64, c_i64,
                                      P]),
    "cg_layernorm_bwd_reduce": (c_int, [P, c_i64, c_i64, c_int, P, P, P, c_int, c_int, P]),
    "cg_layernorm_bwd_reduce_ex": (c_int, [P, c_i64, c_i64, c_int, P, P, P, c_int, c_int, c_int, P]),
    "cg_gemm_workspace": (c_i64, [c_i64, c_i64, c_int]),
    "cg_gemm_colpart_supported": (c_int, [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64]),
    "cg_gemm_relu_bits_supported": (c_int, [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64]),
    "cg_gemm_rowdot_supported": (c_int, [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64]),
    "cg_linear_rows_f32_supported": (c_int, [c_i64, c_i64, c_i64]),
    "cg_decode_qkv_f32": (c_int, [c_i64, c_i64, c_i64, P, c_i64, P, P, c_flt, P, c_i64, P, c_i64, P, c_i64, P, P, P]),
    "cg_linear_rows_f32": (c_int, [c_i64, c_i64, c_i64, P, c_i64, P, P, c_flt, P, c_i64, P, c_int, P, c_i64, P, c_i64, P]),
    "cg_ffn_fwd_f32_supported": (c_int, [c_i64, c_i64, c_i64]),
    "cg_ffn_fwd_f32": (c_int, [c_i64, c_i64, c_i64, P, c_i64, P, P, c_flt, P, c_i64, P, P, c_i64, P, P, c_i64, P,
                               c_i64, P]),
    "cg_gemm_resid_layernorm_supported": (c_int, [c_i64, c_i64, c_i64]),
    "cg_gemm_resid_layernorm": (c_int, [c_i64, c_i64, c_i64, P, c_i64, P, c_i64, P, c_i64, ctypes.POINTER(Epilogue), P, P,
                                        P, P, P, c_flt, P]),
    "cg_flush_deferred": (c_int, [P]),
    "cg_discard_deferred": (c_int, [P, P]),
    "cg_reduce_rows": (c_int, [P, c_i64, c_i64, P, c_int, P]),
    "cg_reduce_rows_ex": (c_int, [P, c_i64, c_i64, P, c_int, c_int, P]),
    "cg_gemm": (c_int, [c_int, c_int, c_int, c_i64, c_i64, c_i64, P, c_i64, P, c_i64, P, c_int, c_i64,
                        ctypes.POINTER(Epilogue), c_int, P, P]),
    "cg_colsum_workspace": (c_i64, [c_i64, c_i64]),
    "cg_colsum": (c_int, [P, c_int, c_i64, c_i64, c_i64, P, c_int, P, P]),
    "cg_attn_fwd": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, P, P, P, c_i64, P, c_i64, P, c_flt, c_dbl, c_u64, P,
                            c_int, P, P]),
    "cg_attn_fwd_premasked": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, P, P, P, c_i64, P, c_i64, P, c_flt, c_dbl,
                                      c_u64, P, c_int, P, P]),
    "cg_attn_dropmask": (c_int, [c_i64, c_i64, c_i64, c_dbl, c_u64, P, c_int, P, P]),
    "cg_layernorm_fwd_attn_dropmask": (c_int, [P, P, P, P, c_int, P, P, c_i64, c_i64, c_flt, c_i64, c_i64, c_i64,
                                               c_dbl, c_u64, P, c_int, P, P]),
    "cg_attn_mask_bytes": (c_i64, [c_i64, c_i64, c_i64]),
    "cg_attn_bwd_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i64]),
    "cg_attn_bwd": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, P, P, P, c_i64, P, c_i64, P, c_i64, P, P, P, P, c_i64,
                            c_flt, c_dbl, c_u64, P, c_int, P, P, P]),
    "cg_attn_bwd_delta": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, P, P, P, c_i64, P, c_i64, P, c_i64, P, P, P, P,
                                  P, c_i64, c_flt, c_dbl, c_u64, P, c_int, P, P, P]),
    "cg_ce_fwd": (c_int, [P, c_i64, c_i64, c_i64, P, P, P, P]),
    "cg_ce_bwd": (c_int, [P, c_i64, c_i64, c_i64, P, P, P, c_flt, P, c_i64, P, P]),
    "cg_head_workspace": (c_i64, [c_i64, c_i64]),
    "cg_head_fwd": (c_int, [P, P, c_i64, P, P, P, P, P, P, c_i64, c_i64, c_i64, P]),
    "cg_head_bwd": (c_int, [P, P, P, P, c_flt, P, P, c_i64, P, c_int, P, c_i64, c_i64, P]),
    "cg_head_bwd_ex": (c_int, [P, P, P, P, c_flt, P, P, c_i64, P, c_int, P, c_i64, c_i64, c_int, P]),
    "cg_decode_window": (c_int, [P, c_i64, c_i64, c_i64, P, P, P]),
    "cg_decode_embed": (c_int, [P, c_i64, P, P, c_i64, P, P, c_i64, P]),
    "cg_decode_kv_append": (c_int, [P, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, P, P, P, P]),
    "cg_decode_attn": (c_int, [P, c_i64, P, P, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, P, c_i64, c_flt, P, c_i64,
                               P]),
    "cg_decode_sample": (c_int, [P, c_i64, c_i64, c_i64, c_int, P, P, P, c_i64, P]),
    "cg_adamw": (c_int, [P, P, P, P, P, c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, P, P]),
    "cg_adamw_defer": (c_int, [P, P, P, P, P, c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, P, P]),
    "cg_adamw_segments": (c_int, [P, P, P, P, P, P, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, P, P]),
    "cg_timing_event_create": (c_int, [ctypes.POINTER(P)]),
    "cg_timing_event_record": (c_int, [P, P]),
    "cg_timing_event_elapsed": (c_int, [P, P, ctypes.POINTER(c_flt)]),
    "cg_timing_event_destroy": (c_int, [P]),
}

_lib = None


def header_symbols():
    """Every cg_* function declared in include/charpt.h."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cg_\w+)\s*\(", src)))


def load():
    """Load (once) and return the ctypes library; raises if it is missing -- no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"charpt: {LIB_PATH} is not built; run `python __graft_entry__.py` (build()) first. "
                           "There is no CPU fallback for the HIP hot path.")
    lib = ctypes.CDLL(LIB_PATH)
    ab = bool(os.environ.get("CHARPT_LIB"))
    for name, (res, args) in _SIGS.items():
        if ab and not hasattr(lib, name):   # an A/B build of an older tree: the entry points it has
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    # CHARPT_TUNING="key=value,key=value": kernel-selection knobs for measurement runs (cg_set_tuning;
    # precision and deferral are per-call flags, not knobs); skip_splitk_reduce (wrong gradients,
    # timing only) additionally needs CHARPT_WHATIF to name it.
    for kv in filter(None, os.environ.get("CHARPT_TUNING", "").split(",")):
        key, _, val = kv.partition("=")
        key = key.strip()
        if key == "skip_splitk_reduce" and "skip_splitk_reduce" not in os.environ.get("CHARPT_WHATIF", ""):
            raise RuntimeError(f"charpt: CHARPT_TUNING may not set {key}")
        check(lib.cg_set_tuning(key.encode(), int(val)), f"cg_set_tuning({key})")
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().cg_last_error_string().decode(errors="replace")
        raise RuntimeError(f"charpt {what} failed (code {rc}): {msg}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def dtype_code(dt):
    if dt == torch.float32:
        return CG_F32
    if dt == torch.bfloat16:
        return CG_BF16
    if dt == torch.int32:
        return CG_BITS   # ReLU keep bits (uint32 words; cg_epilogue_t.aux only)
    raise TypeError(f"charpt: unsupported dtype {dt}")


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
