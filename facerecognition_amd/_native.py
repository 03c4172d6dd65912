"""ctypes binding of the in-tree C-ABI library ``facerecognition_amd/lib/libfrhip.so``.

Every entry point is declared in include/frhip.h.  There is no fallback: if the library is
missing or fails to load, ``lib()`` raises, so the product path can never silently run on the
CPU or on a PyTorch re-implementation.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

LIB_PATH = os.environ.get("FR_LIBFRHIP") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                          "libfrhip.so")  # env: timing-experiment builds
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "frhip.h")

FR_OK = 0
FR_ARCH = {"resnet50_arcface": 0, "iresnet100": 1, "irv1_facenet": 2}
FR_DTYPE_BF16 = 0
FR_DTYPE_F16 = 1
FR_DTYPE_FP8 = 2
FR_DTYPE = {"bf16": FR_DTYPE_BF16, "f16": FR_DTYPE_F16, "fp8": FR_DTYPE_FP8}
FR_IN_U8_NHWC = 0
FR_IN_F32_NCHW = 1
FR_EMBED_RAW = 1
FR_EMBED_ASYNC = 2
FR_ERR_STAGE = -6
FR_TILE_BAND = 7
FR_TILE_IMG28 = 10
FR_TILE_IMG56 = 11
FR_TILE_ROWS = 12
FR_TILE_WRING = 13
FR_TILE_DIRECT = 14
FR_TILE_SMALL = 16
FR_TILE_64x64_S3 = 17
FR_TILE_64x64 = 18
FR_TILE_32x64_S3 = 19
FR_OPT_STAGE = 1
FR_OPT_KEEP_INTERMEDIATES = 2
FR_OPT_MATCH_EXACT = 3
FR_OPT_X3_MIN_ROWS = 4
FR_OPT_STAGE_MIN_FILL = 5
FR_OPT_STAGE_SPIN_LIMIT = 6
FR_OPT_STAGE_VARIANT = 7
FR_OPT_SPLITK_INLAUNCH = 8
FR_OPT_BATCH_INVARIANT = 9
FR_OPT_FUSED_MASK = 10

c_int, c_int64, c_size_t, c_void_p, c_float_p = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p


class FrConvDesc(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("B", c_int), ("H", c_int), ("W", c_int), ("Cx", c_int), ("x_off", c_int), ("Cin", c_int),
        ("w", c_void_p), ("Cout", c_int), ("Kh", c_int), ("Kw", c_int), ("stride_h", c_int), ("stride_w", c_int),
        ("pad_h", c_int), ("pad_w", c_int), ("Npad", c_int), ("Kpad", c_int),
        ("bias", c_void_p), ("act", c_int), ("slope", c_void_p),
        ("res", c_void_p), ("Cres", c_int), ("res_off", c_int),
        ("y", c_void_p), ("Cy", c_int), ("y_off", c_int),
        ("y2", c_void_p), ("Cy2", c_int), ("y2_off", c_int), ("aff_s", c_void_p), ("aff_b", c_void_p),
        ("Ho", c_int), ("Wo", c_int),
        ("split_k", c_int), ("partial", c_void_p), ("dtype", c_int), ("tile", c_int),
        ("bias9", c_void_p),
        ("wscale", c_void_p), ("x_amax", c_void_p), ("y_amax", c_void_p),
    ]


_SIGS = {
    "fr_last_error": (ctypes.c_char_p, []),
    "fr_abi_version": (c_int, []),
    "fr_create": (c_int, [ctypes.POINTER(c_void_p), c_int, c_int, c_int]),
    "fr_destroy": (None, [c_void_p]),
    "fr_load_weights": (c_int, [c_void_p, c_void_p, c_size_t]),
    "fr_reserve": (c_int, [c_void_p, c_int]),
    "fr_embed_dim": (c_int, [c_void_p]),
    "fr_input_size": (c_int, [c_void_p]),
    "fr_embed": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "fr_gallery_set": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int64, c_int]),
    "fr_gallery_rows": (c_int64, [c_void_p]),
    "fr_gallery_write": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int, c_int]),
    "fr_match_topk": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "fr_topk_merge": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "fr_topk_merge_ranks": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "fr_embed_match": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "fr_segment_mean_normalize": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "fr_resize_u8_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "fr_resize_u8": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "fr_warp_affine_u8": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "fr_set_option": (c_int, [c_void_p, c_int, c_int]),
    "fr_get_option": (c_int, [c_void_p, c_int]),
    "fr_debug_match_fallbacks": (c_int, [c_void_p]),
    "fr_debug_stage_timeouts": (c_int, [c_void_p]),
    "fr_debug_stage_reruns": (c_int, [c_void_p]),
    "fr_sync_check": (c_int, [c_void_p, c_void_p]),
    "fr_debug_tensor_count": (c_int, [c_void_p]),
    "fr_debug_tensor_dtype": (c_int, [c_void_p, c_int]),
    "fr_debug_plan": (c_int, [c_void_p, c_int, ctypes.c_char_p, c_size_t]),
    "fr_prof_enable": (c_int, [c_void_p, c_int]),
    "fr_prof_collect": (c_int, [c_void_p]),
    "fr_prof_only": (c_int, [c_void_p, ctypes.c_char_p]),
    "fr_prof_slots": (c_int, [c_void_p, ctypes.c_char_p, c_int]),
    "fr_prof_slot_select": (c_int, [c_void_p, c_int]),
    "fr_prof_slot_ms": (c_int, [c_void_p, c_int, ctypes.POINTER(ctypes.c_float)]),
    "fr_prof_slot_work": (c_int, [c_void_p, c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "fr_prof_get": (c_int, [c_void_p, c_int, ctypes.c_char_p, c_size_t, ctypes.POINTER(ctypes.c_double),
                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "fr_prof_get_bytes": (c_int, [c_void_p, c_int, ctypes.POINTER(ctypes.c_double)]),
    "fr_debug_tensor_name": (ctypes.c_char_p, [c_void_p, c_int]),
    "fr_debug_tensor_shape": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                      ctypes.POINTER(c_int)]),
    "fr_debug_copy_tensor": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "fr_op_conv2d": (c_int, [ctypes.POINTER(FrConvDesc), c_void_p]),
    "fr_area_resample_u8": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "fr_mtcnn_conv": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                              c_void_p, c_void_p]),
    "fr_mtcnn_maxpool": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "fr_mtcnn_dense": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "fr_mtcnn_head": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "fr_nms_host": (c_int, [c_void_p, c_int64, c_void_p, ctypes.c_float, c_int, c_void_p, c_void_p]),
    "fr_op_preprocess": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "fr_op_maxpool": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "fr_op_avgpool": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "fr_op_linear": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                             c_int, c_void_p, c_int, c_void_p]),
}

_lib = None
_lock = threading.Lock()


def header_functions() -> list:
    """Function names declared in include/frhip.h (the ABI contract)."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fr_[a-z0-9_]+)\s*\(", src)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libfrhip.so not built: {LIB_PATH} (run `python -c 'import __graft_entry__ as g; "
                                   f"g.build()'` or `make -C facerecognition_amd/csrc`)")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                if name in _OPTIONAL and not hasattr(L, name):
                    continue  # an older experiment build (FR_LIBFRHIP) without this reporting entry point
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != FR_OK:
        msg = lib().fr_last_error().decode(errors="replace")
        raise RuntimeError(f"frhip {what} failed (rc={rc}): {msg}")


def ptr(t) -> int:
    """Device/host address of a torch tensor (or None → 0)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


_OPTIONAL = {"fr_prof_get_bytes"}  # reporting only: may be absent from older variant builds


def prof_read(handle):
    """fr_prof_collect + fr_prof_get(_bytes) for every class → {name: (total_ms, launches, flops, bytes)}."""
    L = lib()
    n = L.fr_prof_collect(handle)
    check(n if n < 0 else 0, "fr_prof_collect")
    out = {}
    for i in range(n):
        name = ctypes.create_string_buffer(128)
        ms, cnt, fl, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        check(L.fr_prof_get(handle, i, name, 128, ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(fl)), "fr_prof_get")
        if hasattr(L, "fr_prof_get_bytes"):
            check(L.fr_prof_get_bytes(handle, i, ctypes.byref(by)), "fr_prof_get_bytes")
        out[name.value.decode()] = (ms.value, cnt.value, fl.value, by.value)
    return out
