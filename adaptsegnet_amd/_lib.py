"""ctypes binding of the C ABI in include/adaptseg.h (libadaptseg.so, gfx950).

The library is built in-tree by ``make -C adaptsegnet_amd/csrc`` (or
``__graft_entry__.build()``).  There is no fallback: if the shared object is missing or
fails to load, every op raises ``AdaptSegLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# ADAPTSEG_LIBRARY: path of another build of the same library (A/B of two builds on one box,
# experiments/ab_*.sh); default the in-tree build
LIB_PATH = os.environ.get("ADAPTSEG_LIBRARY") or os.path.join(_HERE, "lib", "libadaptseg.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "adaptseg.h")

ADAPTSEG_OK = 0
EPI_LEAKY = 1
EPI_ACCUMULATE = 2
EPI_LEAKY_GRAD = 4
EPI_RESIDUAL = 8
EPI_RELU = 16
EPI_RELU_GRAD = 32
CONV_FWD, CONV_BWD_DATA, CONV_BWD_WEIGHT = 0, 1, 2
MATH_F32, MATH_BF16, MATH_BF16_WIDE, MATH_F32X3, MATH_F32X3_PRESPLIT = 0, 1, 2, 3, 4


class AdaptSegLibraryError(RuntimeError):
    pass


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int), ("c", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
        ("in_stride", ctypes.c_int64 * 4),
        ("k", ctypes.c_int), ("oh", ctypes.c_int), ("ow", ctypes.c_int),
        ("kh", ctypes.c_int), ("kw", ctypes.c_int),
        ("stride", ctypes.c_int), ("nseg", ctypes.c_int),
        ("pad", ctypes.c_int * 4), ("dil", ctypes.c_int * 4),
    ]


class OperandBN(ctypes.Structure):
    """adaptseg_operand_bn (include/adaptseg.h)."""
    _fields_ = [("mean", ctypes.c_void_p), ("invstd", ctypes.c_void_p),
                ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p)]


class BnSumDesc(ctypes.Structure):
    """adaptseg_bnsum_desc (include/adaptseg.h)."""
    _fields_ = [
        ("x", ctypes.c_void_p), ("x_bf16", ctypes.c_void_p),
        ("mean", ctypes.c_void_p), ("invstd", ctypes.c_void_p),
        ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("bits", ctypes.c_void_p), ("mask", ctypes.c_int),
        ("partial", ctypes.c_void_p), ("partial_bytes", ctypes.c_size_t),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float
_SZ = ctypes.c_size_t
_PP = ctypes.POINTER(ctypes.c_void_p)
_DESC = ctypes.POINTER(ConvDesc)

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGS = {
    "adaptseg_last_error": [],
    "adaptseg_version": [],
    "adaptseg_conv2d_workspace_size": [_DESC, _I, ctypes.POINTER(_SZ)],
    "adaptseg_conv2d_kernel_id": [_DESC, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)],
    "adaptseg_conv2d_kernel_id_x": [_DESC, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)],
    "adaptseg_conv2d_copy_operand_only": [_DESC, _I, ctypes.POINTER(_I)],
    "adaptseg_conv2d_operand_bn_ok": [_DESC, _I, ctypes.POINTER(_I)],
    "adaptseg_conv2d_fwd_bnstats_abn": [_DESC, _P, ctypes.POINTER(OperandBN), _PP, _P, _P, _P, _SZ,
                                        ctypes.POINTER(ctypes.c_int), _P, _SZ, _P],
    "adaptseg_conv2d_bwd_weight_abn": [_DESC, _P, _P, ctypes.POINTER(OperandBN), _PP, _I, _P, _SZ, _P],
    "adaptseg_bn_fwd_train_tiles_stats": [_L, _I, _P, _I, _P, _P, _F, _F, _P, _P, _P],
    "adaptseg_conv2d_fwd": [_DESC, _P, _PP, _PP, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_conv2d_bwd_data": [_DESC, _P, _PP, _P, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_conv2d_bwd_weight": [_DESC, _P, _P, _PP, _PP, _I, _P, _SZ, _P],
    "adaptseg_conv2d_wpack_size": [_DESC, _I, ctypes.POINTER(_SZ)],
    "adaptseg_conv2d_wpack": [_DESC, _I, _PP, _P, _SZ, _P],
    "adaptseg_conv2d_fwd_x": [_DESC, _P, _P, _PP, _P, _PP, _P, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_conv2d_fwd_bnstats_x": [_DESC, _P, _P, _PP, _P, _P, _P, _P, _SZ, ctypes.POINTER(ctypes.c_int), _P,
                                      _SZ, _P],
    "adaptseg_conv2d_bwd_data_x": [_DESC, _P, _P, _PP, _P, _P, _P, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_conv2d_bwd_data_xg": [_DESC, _P, _P, _PP, _P, _P, _P, _P, _P, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_conv2d_bwd_weight_x": [_DESC, _P, _P, _P, _P, _PP, _PP, _I, _P, _SZ, _P],
    "adaptseg_conv2d_bnsum_tiles": [_DESC, _I, ctypes.POINTER(_I)],
    "adaptseg_timing_reserve": [_L],
    "adaptseg_conv2d_bwd_data_bnsum": [_DESC, _P, _P, _PP, _P, _P, _P, _P, _P, _P, _I, ctypes.POINTER(BnSumDesc),
                                       ctypes.POINTER(_I), _P, _SZ, _P],
    "adaptseg_bn_bwd_sums": [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _I, _P, _SZ,
                             _P],
    "adaptseg_bn_fwd_train_x": [_L, _I, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_bn_fwd_train_tiles_x": [_L, _I, _P, _I, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _I,
                                      _P],
    "adaptseg_bn_fwd_infer_x": [_L, _I, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _I, _P],
    "adaptseg_bn_fwd_train_xm": [_L, _I, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, _I, _P, _SZ,
                                 _P],
    "adaptseg_bn_fwd_train_tiles_xm": [_L, _I, _P, _I, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P,
                                       _I, _P],
    "adaptseg_bn_fwd_infer_xm": [_L, _I, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P, _I, _P],
    "adaptseg_bn_bwd_x": [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _SZ, _P],
    "adaptseg_bn_bwd_xg": [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _SZ, _P],
    "adaptseg_bn_workspace_size": [_L, _I, ctypes.POINTER(_SZ)],
    "adaptseg_bn_fwd_train": [_L, _I, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_upsample_argmax": [_I, _I, _I, _I, _I, _I, _P, _P, _P],
    "adaptseg_confusion_hist": [_L, _P, _P, _P, _I, _P, _P],
    "adaptseg_bn_fwd_train_tiles": [_L, _I, _P, _I, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _I, _P],
    "adaptseg_conv2d_bnstats_size": [_DESC, ctypes.POINTER(ctypes.c_size_t)],
    "adaptseg_conv2d_bnstats_tiles": [_DESC, ctypes.POINTER(_I)],
    "adaptseg_conv2d_bnstats_tiles_x": [_DESC, _I, ctypes.POINTER(_I)],
    "adaptseg_conv2d_fwd_bnstats": [_DESC, _P, _PP, _P, _P, _SZ, ctypes.POINTER(ctypes.c_int), _P, _SZ, _P],
    "adaptseg_bn_fwd_infer": [_L, _I, _P, _P, _P, _P, _P, _F, _P, _P, _I, _P],
    "adaptseg_bn_bwd": [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _SZ, _P],
    "adaptseg_maxpool2d_fwd": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P],
    "adaptseg_maxpool2d_bwd": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P],
    "adaptseg_maxpool2d_fwd_x": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "adaptseg_maxpool2d_bwd_x": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "adaptseg_upsample_workspace_size": [_I, _I, _I, _I, _I, _I, ctypes.POINTER(_SZ)],
    "adaptseg_upsample_bilinear_fwd": [_I, _I, _I, _I, _I, _I, _P, _P, _P],
    "adaptseg_upsample_bilinear_bwd": [_I, _I, _I, _I, _I, _I, _P, _P, _I, _P, _SZ, _P],
    "adaptseg_softmax_fwd": [_L, _I, _P, _P, _P],
    "adaptseg_softmax_bwd": [_L, _I, _P, _P, _P, _I, _P],
    "adaptseg_ce_workspace_size": [_L, ctypes.POINTER(_SZ)],
    "adaptseg_softmax_ce_fwd": [_L, _I, _P, _P, _I, _P, _P, _P, _SZ, _P],
    "adaptseg_softmax_ce_bwd": [_L, _I, _P, _P, _I, _P, _P, _P, _P, _I, _P],
    "adaptseg_adv_workspace_size": [_L, ctypes.POINTER(_SZ)],
    "adaptseg_adv_loss_fwd": [_L, _P, _F, _I, _P, _P, _SZ, _P],
    "adaptseg_adv_loss_bwd": [_L, _P, _F, _I, _P, _P, _I, _P],
    "adaptseg_sgd_step": [_L, _P, _P, _P, _F, _F, _F, _F, _I, _I, _P],
    "adaptseg_adam_step": [_L, _P, _P, _P, _P, _F, _F, _F, _F, _I, _F, _P],
    "adaptseg_zero": [_P, _SZ, _P],
    "adaptseg_to_nhwc": [_I, _I, _I, _I, ctypes.POINTER(_L), _P, _P, _P],
    "adaptseg_to_nhwc_pad": [_I, _I, _I, _I, ctypes.POINTER(_L), _P, _I, _P, _I, _P],
    "adaptseg_axpy": [_L, _F, _P, _P, _I, _P],
    "adaptseg_add_i64": [_P, _L, _L, _P],
    "adaptseg_preprocess_workspace_size": [_I, _I, _I, _I, _I, ctypes.POINTER(_SZ)],
    "adaptseg_gta5_preprocess": [_I, _I, _I, _I, _I, _P, _F, _F, _F, _P, _P, _P, _P, _P, _SZ, _P],
    "adaptseg_bn_bwd_affine": [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _SZ, _P],
    "adaptseg_up2_relu_cat_fwd": [_I, _I, _I, _I, _I, _P, _P, _P, _P],
    "adaptseg_up2_relu_cat_bwd": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "adaptseg_grid_warp_fwd": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "adaptseg_grid_warp_bwd_workspace_size": [_I, _I, _I, _I, ctypes.POINTER(_SZ)],
    "adaptseg_grid_warp_bwd": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P],
    "adaptseg_conv_set_math": [_I],
    "adaptseg_conv_get_math": [ctypes.POINTER(_I)],
    "adaptseg_conv_set_option": [_I, _I],
    "adaptseg_conv_get_option": [_I, ctypes.POINTER(_I)],
    "adaptseg_splitk_flush": [_P],
    "adaptseg_splitk_pending": [_P, ctypes.POINTER(_I)],
    "adaptseg_stream_create_cu_mask": [_I, _I, ctypes.POINTER(_P)],
    "adaptseg_stream_destroy": [_P],
    "adaptseg_timing_enable": [_I, _I],
    "adaptseg_timing_enable_mem": [_I],
    "adaptseg_timing_read_id": [_I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(_L)],
    "adaptseg_timing_read": [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(_L)],
    "adaptseg_timing_enable_stream": [_I],
    "adaptseg_timing_read_id_stream": [_I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_L)],
}
_RESTYPES = {"adaptseg_last_error": ctypes.c_char_p, "adaptseg_version": ctypes.c_char_p}

_lib = None
_lock = threading.Lock()


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function name declared in include/adaptseg.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(adaptseg_[a-z0-9_]+)\s*\(", text)))


def lib():
    """Load libadaptseg.so (once).  Raises AdaptSegLibraryError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise AdaptSegLibraryError(
                f"{LIB_PATH} not found: build it with `make -C adaptsegnet_amd/csrc` "
                "(the HIP path has no CPU fallback)")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the image
            raise AdaptSegLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        for name, argtypes in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
        return L


def check(status: int, what: str) -> None:
    if status != ADAPTSEG_OK:
        msg = lib().adaptseg_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def ptr_array(ptrs) -> "ctypes.Array":
    arr = (ctypes.c_void_p * 4)()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr
