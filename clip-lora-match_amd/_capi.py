"""ctypes binding of libclm.so (include/clm.h).

The product path has no CPU fallback: if the library or a HIP device is
missing, every call raises. Error codes map to the exception types the
reference raises for the same conditions (ValueError for bad shapes/arguments,
search.py:33-34,83-90; RuntimeError for device failures).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_uint32, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CLM_LIB", os.path.join(_HERE, "libclm.so"))

CLM_OK, CLM_E_ARG, CLM_E_OOM, CLM_E_HIP, CLM_E_STATE, CLM_E_MISSING = 0, -1, -2, -3, -4, -5
CLM_F32, CLM_F16, CLM_BF16, CLM_U8, CLM_I32, CLM_I64 = 0, 1, 2, 3, 4, 5
CLM_ATTN_CAUSAL, CLM_ATTN_Q_LOG2E = 1, 2   # clm_attention_ex flags
CLM_PIX_U8_HWC, CLM_PIX_F32_CHW = 0, 1
CLM_LORA_MERGED, CLM_LORA_UNMERGED = 0, 1
CLM_COMPUTE_MIXED = 0x12   # bf16 vision tower, fp16 text tower (clm.h)
CLM_PAIR_GRAPH = 1
CLM_PAIR_SPLIT_SHIFT = 8


class TowerDesc(ctypes.Structure):
    _fields_ = [("hidden", c_int32), ("layers", c_int32), ("heads", c_int32), ("mlp", c_int32)]


class ModelDesc(ctypes.Structure):
    _fields_ = [
        ("vision", TowerDesc), ("text", TowerDesc),
        ("patch", c_int32), ("image_size", c_int32), ("channels", c_int32),
        ("vocab", c_int32), ("max_pos", c_int32), ("proj_dim", c_int32),
        ("eos_token_id", c_int32), ("ln_eps", c_float),
        ("lora_r", c_int32), ("lora_alpha", c_float), ("lora_targets", c_uint32),
        ("lora_mode", c_int32), ("compute_dtype", c_int32), ("max_batch", c_int32),
        ("mean", c_float * 3), ("std", c_float * 3),
    ]


class ClmError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libclm.so once; raise loudly if it is absent (no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7). Loading torch first
    # makes libclm's DT_NEEDED bind to that same runtime, so torch streams and device
    # pointers are native objects of the runtime libclm calls (one HIP runtime per process).
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libclm.so not found at {LIB_PATH}: build it with `make -C clip-lora-match_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "clm_ctx_create": (c_int, [c_int, POINTER(ModelDesc), POINTER(c_void_p)]),
        "clm_ctx_destroy": (c_int, [c_void_p]),
        "clm_load_tensor": (c_int, [c_void_p, c_char_p, c_void_p, c_int, POINTER(c_int64), c_int]),
        "clm_finalize": (c_int, [c_void_p]),
        "clm_set_lora_enabled": (c_int, [c_void_p, c_int]),
        "clm_set_lora": (c_int, [c_void_p, c_int, ctypes.c_float, c_uint32]),
        "clm_encode_image": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
        "clm_encode_text": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
        "clm_encode_pair": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                    c_int, c_int, c_int, c_void_p]),
        "clm_pair_path": (c_int, [c_void_p]),
        "clm_index_create": (c_int, [c_int, c_int64, c_int, POINTER(c_void_p)]),
        "clm_index_destroy": (c_int, [c_void_p]),
        "clm_index_append": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p]),
        "clm_index_size": (c_int64, [c_void_p]),
        "clm_index_reset": (c_int, [c_void_p]),
        "clm_index_set_offset": (c_int, [c_void_p, c_int64]),
        "clm_index_read": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
        "clm_index_search": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
        "clm_index_stats": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
        "clm_index_stats2": (c_int, [c_void_p, POINTER(c_int64), c_int]),
        "clm_cosine_scores": (c_int, [c_int, c_void_p, c_int64, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
        "clm_topk_merge": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p]),
        "clm_topk_threshold": (c_int, [c_int, c_void_p, c_int64, c_int64, c_int64, c_int, ctypes.c_float, c_int,
                                       c_void_p, c_void_p]),
        "clm_l2_normalize": (c_int, [c_int, c_void_p, c_int64, c_int, c_void_p]),
        "clm_fuse_queries": (c_int, [c_int, c_void_p, ctypes.c_float, c_void_p, ctypes.c_float, c_int64, c_int,
                                     c_void_p, c_void_p]),
        "clm_resize_crop": (c_int, [c_int, c_void_p, POINTER(c_int64), POINTER(c_int32), c_int, c_int, c_void_p,
                                    c_void_p]),
        "clm_synth_images": (c_int, [c_int, ctypes.c_uint64, c_int64, c_int, c_int, c_void_p, c_void_p]),
        "clm_index_has_f32": (c_int, [c_void_p]),
        "clm_index_export": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
        "clm_index_import": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
        "clm_last_error": (c_char_p, []),
        "clm_version": (c_char_p, []),
        "clm_model_desc_size": (c_int32, []),
        "clm_prof_enable": (c_int, [c_void_p, c_int]),
        "clm_gemm": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int,
                             c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
        "clm_gemm_num_configs": (c_int, []),
        "clm_debug_set": (None, [c_int]),
        "clm_attention": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p]),
        "clm_gemm_scores16": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int,
                                      c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
        "clm_attention_ex": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p]),
        "clm_layernorm": (c_int, [c_int, c_int, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_float, c_void_p,
                                  c_int64, c_void_p]),
        "clm_prof_read": (c_int, [c_void_p, c_int, POINTER(ctypes.c_double), POINTER(ctypes.c_double),
                                  POINTER(c_int64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


EXPORTED = (
    "clm_ctx_create", "clm_ctx_destroy", "clm_load_tensor", "clm_finalize", "clm_set_lora_enabled", "clm_set_lora",
    "clm_encode_image", "clm_encode_text", "clm_encode_pair", "clm_pair_path", "clm_index_create", "clm_index_destroy", "clm_index_append",
    "clm_index_size", "clm_index_reset", "clm_index_set_offset", "clm_index_read", "clm_index_search", "clm_index_stats",
    "clm_index_stats2",
    "clm_cosine_scores", "clm_topk_merge", "clm_topk_threshold", "clm_l2_normalize", "clm_fuse_queries", "clm_resize_crop", "clm_synth_images", "clm_index_has_f32", "clm_index_export", "clm_index_import",
    "clm_last_error", "clm_version",
    "clm_model_desc_size", "clm_prof_enable", "clm_prof_read", "clm_gemm", "clm_gemm_num_configs",
    "clm_attention", "clm_attention_ex", "clm_gemm_scores16", "clm_layernorm", "clm_debug_set",
)
CLM_EPI_STORE, CLM_EPI_GELU, CLM_EPI_RESID, CLM_EPI_SCORE = 0, 1, 2, 4
CLM_PROF_GEMM, CLM_PROF_ATTN, CLM_PROF_LN, CLM_PROF_OTHER = 0, 1, 2, 3


def check(rc: int, what: str = "") -> None:
    if rc == CLM_OK:
        return
    msg = lib().clm_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc in (CLM_E_ARG, CLM_E_MISSING):
        raise ValueError(text)
    raise ClmError(f"{text} (code {rc})")


def require_gpu() -> None:
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("clip_lora_match_amd needs an MI355X (gfx950) HIP device; none is visible "
                           "(there is no CPU fallback)")


def ptr(t) -> c_void_p:
    return c_void_p(t.data_ptr())


def stream_of(device) -> c_void_p:
    import torch
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)
