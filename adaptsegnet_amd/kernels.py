"""Tensor-level API of the native ops: allocate outputs, call ``torch.ops.adaptseg.*``.

Activations handed to these functions are contiguous NHWC fp32 CUDA tensors of shape
``[n, h, w, c]`` (the physical layout of a channels_last NCHW tensor) unless a function
says otherwise.  Every call is asynchronous on the current HIP stream; none synchronises.
These are the only functions that launch compute on the hot path, each through one custom
operator of ``adaptsegnet_amd.ops`` (whose CUDA kernel calls the C ABI of include/adaptseg.h)
— there is no CPU or eager-PyTorch fallback, and a missing ``libadaptseg.so`` raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import weakref
from dataclasses import dataclass

import torch

from . import _lib
from . import ops as _ops
from ._lib import (CONV_BWD_DATA, CONV_BWD_WEIGHT, CONV_FWD, EPI_ACCUMULATE, EPI_LEAKY,
                   EPI_LEAKY_GRAD, EPI_RELU, EPI_RELU_GRAD, EPI_RESIDUAL, MATH_BF16, MATH_BF16_WIDE, MATH_F32, MATH_F32X3, MATH_F32X3_PRESPLIT,
                   ConvDesc, check)

__all__ = [
    "ConvGeom", "set_conv_math", "get_conv_math", "MATH_F32", "MATH_BF16", "MATH_BF16_WIDE", "MATH_F32X3", "MATH_F32X3_PRESPLIT", "conv_fwd", "conv_fwd_bnstats", "conv_dgrad", "conv_wgrad", "bn_fwd_train",
    "bn_fwd_train_tiles", "bn_fwd_infer", "bn_bwd",
    "maxpool_fwd", "maxpool_bwd", "upsample_fwd", "upsample_bwd", "softmax_fwd", "softmax_bwd",
    "ce_fwd", "ce_bwd", "adv_fwd", "adv_bwd", "sgd_step", "adam_step", "zero_", "to_nhwc",
    "axpy", "add_i64", "weight_pack_scope", "pack_builds", "pack_count", "clear_weight_packs", "EPI_ACCUMULATE", "EPI_LEAKY", "EPI_LEAKY_GRAD", "EPI_RELU", "EPI_RELU_GRAD", "EPI_RESIDUAL",
]


_OP = _ops.OPS   # torch.ops.adaptseg.*.default: every launch below goes through the dispatcher
_p, _stream, _ws_args, workspace = _ops._p, _ops._stream, _ops._ws_args, _ops.workspace


def _require(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: expected a CUDA (HIP) tensor, got device {t.device}")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{what}: expected float32, got {t.dtype}")


# ---------------------------------------------------------------------------------------
# Convolution
# ---------------------------------------------------------------------------------------
@dataclass(frozen=True)
class ConvGeom:
    """Static geometry of one (possibly multi-segment) convolution."""

    cin: int
    cout: int
    kh: int
    kw: int
    stride: int = 1
    pads: tuple = (0,)
    dils: tuple = (1,)

    @property
    def nseg(self) -> int:
        return len(self.pads)

    def out_hw(self, h: int, w: int):
        p, d = self.pads[0], self.dils[0]
        oh = (h + 2 * p - d * (self.kh - 1) - 1) // self.stride + 1
        ow = (w + 2 * p - d * (self.kw - 1) - 1) // self.stride + 1
        return oh, ow

    def flops(self, n: int, h: int, w: int) -> float:
        oh, ow = self.out_hw(h, w)
        return 2.0 * n * oh * ow * self.cout * self.cin * self.kh * self.kw * self.nseg


def set_conv_math(math: int) -> None:
    """Process-wide conv arithmetic: MATH_F32X3 (default: fp32 through exact three-term bf16
    splits on the bf16 MFMA, fp32-accurate, conv_x3.hpp / conv_x3r.hpp), MATH_F32X3_PRESPLIT (the
    same arithmetic, every product the term-image kernel covers on conv_x3r.hpp, fed bf16 term
    images the BN passes write), MATH_F32 (the fp32-input MFMA
    kernels) or MATH_BF16 (operands rounded to bf16, fp32 accumulate: BASELINE config c5).  Workspace sizes depend on it,
    so the descriptor cache is keyed on it."""
    _ops.set_math(math)


def set_x3h(mode: int) -> None:
    """F32X3: forward (bit 1) / data-gradient (bit 2) / weight-gradient (bit 4) products on the
    256x128x32 tiles with the fp32 operands split in-kernel (igemm_x3h_kernel, igemm_x3hw_kernel)
    instead of the 128x128x16 register-staged kernel (ADAPTSEG_OPT_X3H; initial value from
    ADAPTSEG_X3H)."""
    _ops.set_option(_ops.OPT_X3H, mode)


def get_x3h() -> int:
    return _ops.get_option(_ops.OPT_X3H)


def set_g16_wide(mode) -> None:
    """BF16: bit 1 = forward / data-gradient products with N >= 256 and K >= 2048 on the
    256x256x64 two-stage LDS-DMA tile, bit 2 = weight gradients on the 256x256 tile
    (ADAPTSEG_OPT_G16_WIDE; initial value from ADAPTSEG_G16_WIDE, default 1).  True = 3."""
    _ops.set_option(_ops.OPT_G16_WIDE, 3 if mode is True else int(mode))


def get_g16_wide() -> int:
    return _ops.get_option(_ops.OPT_G16_WIDE)


def get_conv_math() -> int:
    m = ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv_get_math(ctypes.byref(m)), "conv_get_math")
    return m.value


def _desc(g: ConvGeom, n, h, w, strides):
    return _ops.conv_desc(n, g.cin, h, w, strides, g.cout, g.kh, g.kw, g.stride, g.pads, g.dils)


# ---------------------------------------------------------------------------------------
# Weight packs, built once per training step
# ---------------------------------------------------------------------------------------
class _PackCache:
    """Caller-owned weight packs (adaptseg_conv2d_wpack) of the F32X3 / bf16 forward and
    data-gradient kernels.  Active only inside weight_pack_scope(); every pack built inside a
    scope is stale once the outermost scope exits (the next use rebuilds it in place).

    Packs are held per weight TENSOR (keyed by the first weight of the product, dropped by a
    weakref finalizer on it), so they live exactly as long as the model that owns the weights: dropping a model
    (a test, an eval loop, a re-created trainer) frees its packs.  Persistent cost while a model
    lives: F32X3 forward + data-gradient packs are 3 bf16 terms each = 12 B per weight (DeeplabMulti
    ~0.5 GB), bf16 packs 4 B per weight.  clear_weight_packs() drops every pack at once."""

    def __init__(self):
        self.depth = 0       # weight_pack_scope nesting
        self.epoch = 0       # bumped when the outermost scope exits
        # id(first weight) -> {(weight data_ptrs, geometry, op, math): [pack buffer (uint8), epoch
        # built]}; a weakref.finalize on the weight drops its entry (tensors compare elementwise,
        # so they cannot key a WeakKeyDictionary)
        self.entries = {}
        # id(first weight) -> its weakref.finalize: ONE per weight, kept across
        # clear_weight_packs() and reused while alive (a long-lived Parameter gains no more)
        self.finalizers = {}
        # (geometry, op, math, NHWC input?) -> pack bytes (0: the kernel reads none)
        self.sizes = {}
        self.builds = 0      # packs built (tests)

    def _drop(self, wid):
        self.entries.pop(wid, None)
        self.finalizers.pop(wid, None)

    def track(self, weight):
        """The per-weight pack dict of ``weight`` (created on first use).  Entries are keyed by
        id(weight); the inner keys add every segment's data_ptr, so a product over several
        weights (the ASPP's four) is found through its first weight and rebuilt if any segment
        moved."""
        wid = id(weight)
        per = self.entries.get(wid)
        if per is None:
            per = self.entries[wid] = {}
            f = self.finalizers.get(wid)
            if f is None or not f.alive:
                self.finalizers[wid] = weakref.finalize(weight, self._drop, wid)
        return per


_PACKS = _PackCache()


@contextlib.contextmanager
def weight_pack_scope():
    """Inside the scope each conv's weight pack is built ONCE and reused by every forward /
    data-gradient call on the same weights (a c2 step calls each G conv's forward twice and
    each D conv's three times); leaving the outermost scope marks every pack stale.  The caller
    promises not to write the weights inside it: AdaptSegTrainer.step wraps its step body, whose
    optimiser launches (train_gta2cityscapes_multi.py:532-540) follow the step's last conv.  A
    weight write between steps (load_state_dict, .data, a user's optimiser) is therefore always
    seen by the next step's packs.  Outside any scope every call packs for itself."""
    _PACKS.depth += 1
    try:
        yield
    finally:
        _PACKS.depth -= 1
        if _PACKS.depth == 0:
            _PACKS.epoch += 1


def pack_builds() -> int:
    """Number of weight packs built through the cache so far (tests)."""
    return _PACKS.builds


def pack_count() -> int:
    """Weight packs currently held (tests: they go with their weights)."""
    return sum(len(v) for v in list(_PACKS.entries.values()))


def clear_weight_packs() -> None:
    """Drop every cached weight pack (their device memory returns to the caching allocator)."""
    _PACKS.entries.clear()


def _wpack(g, n, h, w, strides, weights, op):
    """The cached weight pack for this product inside a weight_pack_scope, else None."""
    if _PACKS.depth == 0:
        return None
    if not _aligned16(*weights):   # the pack kernels read float4 rows; the conv plan falls back
        return None
    math = _ops._CONV_MATH[0]
    skey = (g, op, math, strides[1] == 1)   # the plan (and its pack) depends on the input layout
    size = _PACKS.sizes.get(skey)
    if size is None:
        d = _desc(g, n, h, w, tuple(strides))[0]
        b = ctypes.c_size_t(0)
        check(_lib.lib().adaptseg_conv2d_wpack_size(ctypes.byref(d), op, ctypes.byref(b)), "conv2d_wpack_size")
        size = _PACKS.sizes[skey] = b.value
    if size == 0:
        return None
    per = _PACKS.track(weights[0])
    key = (tuple(t.data_ptr() for t in weights), g, op, math)
    e = per.get(key)
    if e is None or e[0].numel() < size:
        e = per[key] = [torch.empty(size, dtype=torch.uint8, device=weights[0].device), -1]
    if e[1] != _PACKS.epoch:
        _OP.conv2d_wpack(list(weights), e[0], (n, g.cin, h, w), tuple(strides), _wshape(g), g.stride, g.pads,
                         g.dils, op)
        e[1] = _PACKS.epoch
        _PACKS.builds += 1
    return e[0]


def nhwc_strides(n, h, w, c):
    """(n, c, h, w) element strides of a contiguous NHWC buffer."""
    return (h * w * c, 1, w * c, c)


def _wshape(g: ConvGeom):
    return (g.cout, g.cin, g.kh, g.kw)


def conv_fwd(g: ConvGeom, x: torch.Tensor, n: int, h: int, w: int, weights, biases=None,
             strides=None, out=None, res=None, flags: int = 0, xb=None, bf16_out: bool = False,
             bf16_only: bool = False):
    """y[n,oh,ow,cout] = sum_seg conv(x, w_seg) + sum_seg b_seg (+res) (EPI_LEAKY / EPI_RELU).
    xb: optional bf16 copy of x (contiguous NHWC) for the bf16 conv math (bn_* ``bf16_out``).
    bf16_out: also return a bf16 copy of y written by the epilogue -> (y, yb).
    bf16_only: y stored as bf16 only (bf16 activation storage): returns the bf16 tensor."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    oh, ow = g.out_hw(h, w)
    dev = (x if x is not None else xb).device
    if bf16_only:
        outb = torch.empty((n, oh, ow, g.cout), device=dev, dtype=torch.bfloat16)
        wp = _wpack(g, n, h, w, strides, weights, CONV_FWD)
        _OP.conv2d_fwd(x, xb, list(weights), wp, list(biases) if biases is not None else [], res, None, outb,
                       (n, g.cin, h, w), strides, _wshape(g), g.stride, g.pads, g.dils,
                       flags | (EPI_RESIDUAL if res is not None else 0))
        return outb
    if out is None:
        out = torch.empty((n, oh, ow, g.cout), device=dev, dtype=torch.float32)
    if res is not None:
        flags |= EPI_RESIDUAL
    outb = _bf16_like(out, bf16_out)
    wp = _wpack(g, n, h, w, strides, weights, CONV_FWD)
    _OP.conv2d_fwd(x, xb, list(weights), wp, list(biases) if biases is not None else [], res, out, outb,
                   (n, g.cin, h, w), strides, _wshape(g), g.stride, g.pads, g.dils, flags)
    return (out, outb) if bf16_out else out


def conv_bnstats_tiles(g: ConvGeom, n: int, h: int, w: int, strides, with_copy: bool = False) -> int:
    d = _desc(g, n, h, w, tuple(strides))[0]
    nt = ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv2d_bnstats_tiles_x(ctypes.byref(d), 1 if with_copy else 0, ctypes.byref(nt)),
          "conv2d_bnstats_tiles")
    return nt.value


def conv_fwd_bnstats(g: ConvGeom, x: torch.Tensor, n: int, h: int, w: int, weights, strides=None, xb=None,
                     bf16_only: bool = False):
    """y = conv(x, w) plus the per-row-tile BatchNorm statistics of y when the kernel can
    produce them: returns (y, (stats, ntiles)) or (y, None).  bf16_only: y is stored as bf16
    only (bf16 activation storage, config c5; the statistics still come from the fp32
    accumulators)."""
    strides = tuple(strides or nhwc_strides(n, h, w, g.cin))
    nt = conv_bnstats_tiles(g, n, h, w, strides, with_copy=xb is not None and _aligned16(xb))
    # the tile count is planned for 16-byte aligned operands; an unaligned view (a storage
    # offset) takes a kernel without fused statistics, so plan the plain forward for it
    if nt == 0 or not _aligned16(x, *weights):
        return conv_fwd(g, x, n, h, w, weights, strides=strides, xb=xb, bf16_only=bf16_only), None
    oh, ow = g.out_hw(h, w)
    dev = (x if x is not None else xb).device
    shape = (n, oh, ow, g.cout)
    out = None if bf16_only else torch.empty(shape, device=dev, dtype=torch.float32)
    outb = torch.empty(shape, device=dev, dtype=torch.bfloat16) if bf16_only else None
    stats = torch.empty(nt * (1 + 2 * g.cout), device=dev, dtype=torch.float32)
    wp = _wpack(g, n, h, w, strides, weights, CONV_FWD)
    _OP.conv2d_fwd_bnstats(x, xb, list(weights), wp, out, outb, stats, (n, g.cin, h, w), strides, _wshape(g),
                           g.stride, g.pads, g.dils, nt)
    return (outb if bf16_only else out), (stats, nt)


def _aligned16(*ts) -> bool:
    return all(t is None or t.data_ptr() % 16 == 0 for t in ts)


@dataclass
class OperandBN:
    """A train-mode BatchNorm + ReLU folded into its consumer conv's operand gather
    (adaptseg_operand_bn): the conv reads relu((x_pre - mean) * invstd * weight + bias), bitwise
    the BN apply pass's output, which is never written."""
    mean: torch.Tensor
    invstd: torch.Tensor
    weight: torch.Tensor | None
    bias: torch.Tensor | None


def operand_bn_ok(g: ConvGeom, n: int, h: int, w: int, op: int) -> bool:
    """Product ``op`` of this conv (contiguous NHWC input) has an operand-BN kernel (the x3h
    forward, the register-staged F32X3 weight gradient; BN of <= 512 channels)."""
    return _ops.operand_bn_ok((n, g.cin, h, w), nhwc_strides(n, h, w, g.cin), _wshape(g), g.stride, g.pads, g.dils,
                              op)


def conv_fwd_bnstats_abn(g: ConvGeom, x_pre: torch.Tensor, abn: OperandBN, n: int, h: int, w: int, weights):
    """conv_fwd_bnstats of relu(bn(x_pre)) with the BN folded into the gather: (y, (stats, ntiles))."""
    strides = nhwc_strides(n, h, w, g.cin)
    nt = conv_bnstats_tiles(g, n, h, w, strides)
    if nt == 0 or not _aligned16(x_pre, *weights):
        raise RuntimeError("conv_fwd_bnstats_abn: no fused-statistics plan for this product / unaligned operand")
    oh, ow = g.out_hw(h, w)
    out = torch.empty((n, oh, ow, g.cout), device=x_pre.device, dtype=torch.float32)
    stats = torch.empty(nt * (1 + 2 * g.cout), device=x_pre.device, dtype=torch.float32)
    wp = _wpack(g, n, h, w, strides, weights, CONV_FWD)
    _OP.conv2d_fwd_bnstats_abn(x_pre, abn.mean, abn.invstd, abn.weight, abn.bias, list(weights), wp, out, stats,
                               (n, g.cin, h, w), strides, _wshape(g), g.stride, g.pads, g.dils, nt)
    return out, (stats, nt)


def conv_wgrad_abn(g: ConvGeom, dy: torch.Tensor, x_pre: torch.Tensor, abn: OperandBN, n: int, h: int, w: int, dws,
                   accumulate: bool = True) -> None:
    """conv_wgrad with the x operand relu(bn(x_pre)) (no bias gradient)."""
    _OP.conv2d_bwd_weight_abn(dy, x_pre, abn.mean, abn.invstd, abn.weight, abn.bias, list(dws), (n, g.cin, h, w),
                              nhwc_strides(n, h, w, g.cin), _wshape(g), g.stride, g.pads, g.dils,
                              EPI_ACCUMULATE if accumulate else 0)


def conv_bnsum_tiles(g: ConvGeom, n: int, h: int, w: int, with_copy: bool = False) -> int:
    """Row tiles of the fused BN backward sums of this data gradient (0: its plan cannot fuse them)."""
    d = _desc(g, n, h, w, nhwc_strides(n, h, w, g.cin))[0]
    nt = ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv2d_bnsum_tiles(ctypes.byref(d), 1 if with_copy else 0, ctypes.byref(nt)),
          "conv2d_bnsum_tiles")
    return nt.value


@dataclass
class BnSum:
    """The BN whose incoming gradient a data gradient produces (conv_dgrad ``bnsum``): its input
    x (fp32 or bf16, [.., C]), saved mean / invstd, affine weight / bias, and the mask its
    backward applies — BNSUM_RELU_X (ReLU recomputed from x), BNSUM_BITS (``bits``) or BNSUM_NONE."""
    x: torch.Tensor
    mean: torch.Tensor
    invstd: torch.Tensor
    weight: torch.Tensor | None
    bias: torch.Tensor | None
    mask: int
    bits: torch.Tensor | None = None


BNSUM_NONE, BNSUM_RELU_X, BNSUM_BITS = 0, 1, 2


def conv_dgrad(g: ConvGeom, dy: torch.Tensor, n: int, h: int, w: int, weights, out=None,
               res=None, aux=None, flags: int = 0, dyb=None, bf16_out: bool = False, bf16_only: bool = False,
               resbits=None, bnsum: BnSum | None = None):
    """dx[n,h,w,cin] (+)= conv_transpose(dy, w) (+res) (*leaky'(aux), or relu'(aux) with EPI_RELU_GRAD).
    bf16_out: also return a bf16 copy of dx written by the epilogue -> (dx, dxb).
    bf16_only (or a bf16 ``out``): dx stored in bf16 only — bf16 gradient storage (BF16 maths);
    ``res`` may be fp32 or bf16 (adaptseg_conv2d_bwd_data_xg).  resbits: a mask bitmap
    (mask_bits_like) gating res element-wise.
    bnsum: also compute, in the epilogue, the backward sums of that BN over dx — then the result
    is (the usual return value, (partial, ntiles) or None when the plan cannot fuse them)."""
    low = bf16_only or (out is not None and out.dtype == torch.bfloat16)
    dev = (dy if dy is not None else dyb).device
    if out is None:
        out = torch.empty((n, h, w, g.cin), device=dev, dtype=torch.bfloat16 if low else torch.float32)
    if res is not None:
        flags |= EPI_RESIDUAL
    if aux is not None and not flags & EPI_RELU_GRAD:   # the same gating rule in both storages
        # (no caller passes aux to the bf16-storage path; the kernel would apply LeakyReLU' there)
        assert not low, "conv_dgrad: aux with bf16 gradient storage is not a supported combination"
        flags |= EPI_LEAKY_GRAD
    outb = None if low else _bf16_like(out, bf16_out)
    dx, dxb = (None, out) if low else (out, outb)
    wp = _wpack(g, n, h, w, nhwc_strides(n, h, w, g.cin), weights, CONV_BWD_DATA)
    ret = out if (low or not bf16_out) else (out, outb)
    nt = 0
    # the launch-time conditions of the fused sums (adaptseg_conv2d_bwd_data_bnsum): 16-B aligned
    # operands (an unaligned dY or weight downgrades the plan; the BN vectors and its fp32 x are read
    # as float4) and C % 4 == 0 — otherwise the unfused call, and bn_bwd runs its own reduction
    if (bnsum is not None and aux is None and g.cin % 4 == 0 and _aligned16(dy, *weights) and
            _aligned16(bnsum.mean, bnsum.invstd, bnsum.weight, bnsum.bias) and
            (bnsum.x is None or bnsum.x.dtype != torch.float32 or _aligned16(bnsum.x))):
        nt = conv_bnsum_tiles(g, n, h, w, with_copy=dyb is not None and _aligned16(dyb))
    if nt == 0:
        _OP.conv2d_bwd_data(dy, dyb, list(weights), wp, res, resbits, aux, dx, dxb, (n, g.cin, h, w), _wshape(g),
                            g.stride, g.pads, g.dils, flags)
        return ret if bnsum is None else (ret, None)
    partial = torch.empty(2 * g.cin * nt, device=dev, dtype=torch.float32)
    b = bnsum
    _OP.conv2d_bwd_data_bnsum(dy, dyb, list(weights), wp, res, resbits, dx, dxb, (n, g.cin, h, w), _wshape(g),
                              g.stride, g.pads, g.dils, flags, b.x, b.mean, b.invstd, b.weight, b.bias, b.bits,
                              int(b.mask), partial, nt)
    return ret, (partial, nt)


def conv_wgrad(g: ConvGeom, dy: torch.Tensor, x: torch.Tensor, n: int, h: int, w: int, dws,
               dbs=None, strides=None, accumulate: bool = True, dyb=None, xb=None, defer: bool = False) -> None:
    """dw_seg (+)= sum dy (x) x_gathered ; db_seg (+)= sum dy.  dyb / xb: bf16 copies of the
    operands (bf16 conv math): the LDS-DMA weight-gradient kernel uses them together; the
    tap-GEMM (ASPP) path uses xb alone (its dY operand is its own scattered buffer).
    defer: a split-K sum into dw is left pending on the current stream until splitk_flush()
    (adaptseg.h ADAPTSEG_WGRAD_DEFER_SUM); dw must not be read before it."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    flags = (EPI_ACCUMULATE if accumulate else 0) | (_ops.WGRAD_DEFER_SUM if defer else 0)
    _OP.conv2d_bwd_weight(dy, dyb, x, xb, list(dws), list(dbs) if dbs is not None else [], (n, g.cin, h, w), strides,
                          _wshape(g), g.stride, g.pads, g.dils, flags)


def splitk_flush() -> None:
    """Launch the split-K sums deferred on the current stream (conv_wgrad(..., defer=True))."""
    _ops.splitk_flush()


def splitk_pending() -> int:
    return _ops.splitk_pending()


def stream_create_cu_mask(k: int, d: int) -> int:
    """A HIP stream on the CUs i with i % d < k (adaptseg_stream_create_cu_mask); returns the
    handle (wrap it with torch.cuda.ExternalStream)."""
    h = ctypes.c_void_p(0)
    _lib.check(_lib.lib().adaptseg_stream_create_cu_mask(int(k), int(d), ctypes.byref(h)), "stream_create_cu_mask")
    return h.value


# ---------------------------------------------------------------------------------------
# BatchNorm (x as [rows, C])
# ---------------------------------------------------------------------------------------
def copies_are_terms() -> bool:
    """Under the F32X3 maths an operand copy holds the three bf16 terms of an fp32 tensor
    [..., C], pixel-interleaved as [..., 3, C] (adaptseg.h: the _x forms' copies); under BF16 it
    is one bf16 (RNE) image of the same shape."""
    return _ops._CONV_MATH[0] in (MATH_F32X3, MATH_F32X3_PRESPLIT)


def _bf16_like(t, want):
    if not want:
        return None
    shape = tuple(t.shape[:-1]) + ((3,) if copies_are_terms() else ()) + (t.shape[-1],)
    return torch.empty(shape, device=t.device, dtype=torch.bfloat16)


def _f32_like(t):
    return torch.empty(t.shape, device=t.device, dtype=torch.float32)


def mask_bits_like(t):
    """A ReLU mask bitmap for a [..., C] activation (C % 32 == 0): int32 [rows, C / 32], bit c % 32
    of word (row, c / 32) = element (row, c) > 0 (written by the bn_fwd_* ``ybits`` argument)."""
    c = t.shape[-1]
    if c % 32:
        raise RuntimeError(f"mask_bits_like: C must be a multiple of 32, got {c}")
    return torch.empty((t.numel() // c, c // 32), device=t.device, dtype=torch.int32)


def bn_fwd_train(x, weight, bias, running_mean, running_var, momentum, eps, res=None,
                 relu=True, out=None, bf16_out=False, fp32_out=True, ybits=None):
    """bf16_out: also return a bf16 (RNE) copy of y, the operand of a bf16-math conv: (y, mean,
    invstd, yb).  fp32_out=False (with bf16_out): only the copy is written, y is None.
    x / res may be bf16 tensors (bf16 activation storage), both or neither."""
    c = x.shape[-1]
    y = (_f32_like(x) if out is None else out) if (fp32_out or not bf16_out) else None
    yb = _bf16_like(x, bf16_out)
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    invstd = torch.empty(c, device=x.device, dtype=torch.float32)
    _OP.bn_fwd_train(x, weight, bias, running_mean, running_var, res, y, yb, ybits, mean, invstd, float(momentum),
                     float(eps), int(relu))
    return (y, mean, invstd, yb) if bf16_out else (y, mean, invstd)


def bn_fwd_train_tiles(x, tiles, weight, bias, running_mean, running_var, momentum, eps, res=None,
                       relu=True, out=None, bf16_out=False, fp32_out=True, ybits=None):
    """bn_fwd_train whose statistics come from conv_fwd_bnstats's row tiles.  ybits: the caller's
    mask_bits_like(x) bitmap to fill with y's ReLU mask (or None)."""
    stats, ntiles = tiles
    c = x.shape[-1]
    y = (_f32_like(x) if out is None else out) if (fp32_out or not bf16_out) else None
    yb = _bf16_like(x, bf16_out)
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    invstd = torch.empty(c, device=x.device, dtype=torch.float32)
    _OP.bn_fwd_train_tiles(x, stats, int(ntiles), weight, bias, running_mean, running_var, res, y, yb, ybits, mean,
                           invstd, float(momentum), float(eps), int(relu))
    return (y, mean, invstd, yb) if bf16_out else (y, mean, invstd)


def bn_fwd_train_tiles_stats(x, tiles, running_mean, running_var, momentum, eps):
    """The statistics half of bn_fwd_train_tiles alone (x: the BN input, for its shape): returns
    (mean, invstd); for a BN folded into its consumer conv (OperandBN)."""
    stats, ntiles = tiles
    c = x.shape[-1]
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    invstd = torch.empty(c, device=x.device, dtype=torch.float32)
    _OP.bn_fwd_train_tiles_stats(stats, int(ntiles), x.numel() // c, c, running_mean, running_var, mean, invstd,
                                 float(momentum), float(eps))
    return mean, invstd


def bn_fwd_infer(x, weight, bias, running_mean, running_var, eps, res=None, relu=True, out=None,
                 bf16_out=False, fp32_out=True, ybits=None):
    y = (_f32_like(x) if out is None else out) if (fp32_out or not bf16_out) else None
    yb = _bf16_like(x, bf16_out)
    _OP.bn_fwd_infer(x, weight, bias, running_mean, running_var, res, y, yb, ybits, float(eps), int(relu))
    return (y, yb) if bf16_out else y


def bn_bwd(dy, y, x, weight, mean, invstd, relu=True, dx=None, dres=None, train=True, bias=None,
           bf16_out=False, fp32_out=True, dybits=None, sums=None):
    """dx = BN-backward(g), g = dy*[y>0] if relu; dres receives g.  dx/dres may alias dy.
    y=None with relu (train mode): the mask is recomputed from x, weight and bias.
    dybits: a mask bitmap (mask_bits_like) applied to dy first, g = dy * bit.
    bf16_out: return (dx, dxb) with a bf16 (RNE) copy of dx (a bf16-math data-gradient operand);
    fp32_out=False (with bf16_out): only the copy is written, dx is None.
    sums: (partial, ntiles) from conv_dgrad(bnsum=...) over this dy (train mode): the reduction
    pass is skipped."""
    if not (fp32_out or not bf16_out):
        dx = None
    elif dx is None:
        dx = torch.empty(dy.shape, device=dy.device, dtype=torch.float32)
    dxb = _bf16_like(dy, bf16_out)
    if sums is not None and train:
        _OP.bn_bwd_sums(dy, dybits, y, x, weight, bias, mean, invstd, dx, dxb, dres, int(relu), sums[0], int(sums[1]))
    else:
        _OP.bn_bwd(dy, dybits, y, x, weight, bias, mean, invstd, dx, dxb, dres, int(relu), bool(train))
    return (dx, dxb) if bf16_out else dx


ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2   # the BN entry points' activation codes


def bn_bwd_affine(dy, y, x, weight, bias, mean, invstd, act, dweight=None, dbias=None, dx=None):
    """Train-mode BN backward with trainable affine parameters: dx, plus dweight/dbias
    accumulated (sum g*xhat, sum g).  act: ACT_NONE / ACT_RELU / ACT_LEAKY (mask from y, or
    from x when y is None).  dx may alias dy."""
    if dx is None:
        dx = torch.empty_like(dy)
    _OP.bn_bwd_affine(dy, y, x, weight, bias, mean, invstd, dx, int(act), dweight, dbias)
    return dx


# ---------------------------------------------------------------------------------------
# Warper: decoder input (ReLU + x2 upsample + skip concat) and the prediction warp
# ---------------------------------------------------------------------------------------
def up2_relu_cat_fwd(s, d):
    """NHWC up2(relu(cat(s, d))) at twice the resolution; s may be None."""
    n, h, w, cd = d.shape
    cs = 0 if s is None else s.shape[-1]
    out = torch.empty((n, 2 * h, 2 * w, cs + cd), device=d.device, dtype=torch.float32)
    _OP.up2_relu_cat_fwd(s, d, out)
    return out


def up2_relu_cat_bwd(s, d, dout, ds=None, dd=None):
    """(ds, dd) = masked split of up2^T(dout); ds is None when s is None."""
    if dd is None:
        dd = torch.empty_like(d)
    if s is not None and ds is None:
        ds = torch.empty_like(s)
    _OP.up2_relu_cat_bwd(s, d, dout, ds, dd)
    return ds, dd


def grid_warp_fwd(flow, x1, x2):
    """ResNetMulti.warp of both heads (NHWC [n,h,w,c]; x1 may be None) by one NHWC warp field."""
    y1 = None if x1 is None else torch.empty_like(x1)
    y2 = torch.empty_like(x2)
    _OP.grid_warp_fwd(flow, x1, x2, y1, y2)
    return y1, y2


def grid_warp_bwd(flow, x1, x2, dy1, dy2, need_dflow=True, need_dx1=True, need_dx2=True):
    """-> (dflow, dx1, dx2); entries not requested (or without their dy) are None."""
    dflow = torch.empty_like(flow) if need_dflow else None
    dx1 = torch.empty_like(dy1) if (need_dx1 and dy1 is not None) else None
    dx2 = torch.empty_like(dy2) if (need_dx2 and dy2 is not None) else None
    _OP.grid_warp_bwd(flow, x1 if dy1 is not None else None, x2 if dy2 is not None else None, dy1, dy2,
                      dflow, dx1, dx2)
    return dflow, dx1, dx2


# ---------------------------------------------------------------------------------------
# Pooling / interpolation / softmax / losses
# ---------------------------------------------------------------------------------------
def maxpool_fwd(x, k=3, s=2, p=1, terms=False):
    """-> (y, argmax), or (y, argmax, y's F32X3 term images [n, oh, ow, 3, c]) with ``terms``."""
    n, h, w, c = x.shape
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    y = torch.empty((n, oh, ow, c), device=x.device, dtype=torch.float32)
    am = torch.empty((n, oh, ow, c), device=x.device, dtype=torch.uint8)
    yt = torch.empty((n, oh, ow, 3, c), device=x.device, dtype=torch.bfloat16) if terms else None
    _OP.maxpool2d_fwd(x, y, am, yt, k, s, p)
    return (y, am, yt) if terms else (y, am)


def maxpool_bwd(dy, am, h, w, k=3, s=2, p=1, terms=False):
    """-> dx, or (dx, dx's F32X3 term images [n, h, w, 3, c]) with ``terms``."""
    n, oh, ow, c = dy.shape
    dx = torch.empty((n, h, w, c), device=dy.device, dtype=torch.float32)
    dxt = torch.empty((n, h, w, 3, c), device=dy.device, dtype=torch.bfloat16) if terms else None
    _OP.maxpool2d_bwd(dy, am, dx, dxt, k, s, p)
    return (dx, dxt) if terms else dx


def upsample_fwd(x, oh, ow):
    n, h, w, c = x.shape
    y = torch.empty((n, oh, ow, c), device=x.device, dtype=torch.float32)
    _OP.upsample_bilinear_fwd(x, y)
    return y


def upsample_bwd(dy, h, w, out=None, accumulate=False):
    n, oh, ow, c = dy.shape
    if out is None:
        out = torch.empty((n, h, w, c), device=dy.device, dtype=torch.float32)
    _OP.upsample_bilinear_bwd(dy, out, bool(accumulate))
    return out


def softmax_fwd(x):
    y = torch.empty_like(x)
    _OP.softmax_fwd(x, y)
    return y


def softmax_bwd(y, dy, out=None, accumulate=False):
    if out is None:
        out = torch.empty_like(y)
    _OP.softmax_bwd(y, dy, out, bool(accumulate))
    return out


def ce_fwd(logits, labels, ignore=255, class_weight=None):
    """Returns a 2-element device tensor [loss, denominator]."""
    out = torch.empty(2, device=logits.device, dtype=torch.float32)
    _OP.softmax_ce_fwd(logits, labels, int(ignore), class_weight, out)
    return out


def ce_bwd(logits, labels, out2, grad_loss, ignore=255, class_weight=None, dl=None,
           accumulate=False):
    if dl is None:
        dl = torch.empty_like(logits)
    _OP.softmax_ce_bwd(logits, labels, out2, grad_loss, int(ignore), class_weight, dl, bool(accumulate))
    return dl


def adv_fwd(x, target: float, kind: int):
    loss = torch.empty(1, device=x.device, dtype=torch.float32)
    _OP.adv_loss_fwd(x, float(target), int(kind), loss)
    return loss


def adv_bwd(x, target: float, kind: int, grad_loss, dx=None, accumulate=False):
    if dx is None:
        dx = torch.empty_like(x)
    _OP.adv_loss_bwd(x, float(target), int(kind), grad_loss, dx, bool(accumulate))
    return dx


# ---------------------------------------------------------------------------------------
# Optimisers and plumbing
# ---------------------------------------------------------------------------------------
def sgd_step(param, grad, mom, lr, momentum, weight_decay, grad_scale=1.0, multiplicity=1,
             first_step=False):
    _OP.sgd_step(param, grad, mom, float(lr), float(momentum), float(weight_decay), float(grad_scale),
                 int(multiplicity), bool(first_step))


def adam_step(param, grad, m, v, lr, beta1, beta2, eps, step, grad_scale=1.0):
    _OP.adam_step(param, grad, m, v, float(lr), float(beta1), float(beta2), float(eps), int(step),
                  float(grad_scale))


def zero_(t: torch.Tensor) -> torch.Tensor:
    _OP.zero(t)
    return t


def to_nhwc(t: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor (any strides) -> contiguous NHWC buffer [n, h, w, c]."""
    _require(t, "to_nhwc")
    n, c, h, w = t.shape
    out = torch.empty((n, h, w, c), device=t.device, dtype=torch.float32)
    _OP.to_nhwc(t, out)
    return out


def axpy(alpha, src, dst, accumulate=True):
    _OP.axpy(float(alpha), src, dst, bool(accumulate))
    return dst


def add_i64(t: torch.Tensor, v: int = 1):
    _OP.add_i64(t, int(v))


def to_nhwc_pad(t: torch.Tensor, c_dst: int, out: torch.Tensor | None = None,
                accumulate: bool = False) -> torch.Tensor:
    """NCHW-shaped tensor [n, c, h, w] (any strides) -> NHWC buffer [n, h, w, c_dst], channels
    c..c_dst-1 zero (out += with accumulate: the first c channels of a padded gradient fold
    back into an unpadded one)."""
    _require(t, "to_nhwc_pad")
    n, c, h, w = t.shape
    if out is None:
        out = torch.empty((n, h, w, c_dst), device=t.device, dtype=torch.float32)
    if tuple(out.shape) != (n, h, w, c_dst) or not out.is_contiguous() or c_dst < c:
        raise RuntimeError(f"to_nhwc_pad: out must be a contiguous [{n}, {h}, {w}, {c_dst}] buffer, c_dst >= {c}")
    _OP.to_nhwc_pad(t, out, bool(accumulate))
    return out


def nhwc_view(t: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor -> its NHWC buffer (no copy if channels_last-contiguous)."""
    if t.dim() == 4 and t.permute(0, 2, 3, 1).is_contiguous():
        return t.permute(0, 2, 3, 1)
    return to_nhwc(t)


def as_nchw(t: torch.Tensor) -> torch.Tensor:
    """NHWC buffer [n, h, w, c] -> NCHW-shaped channels_last view."""
    return t.permute(0, 3, 1, 2)


# ---------------------------------------------------------------------------------------
# Live kernel timing (bench.py roofline)
# ---------------------------------------------------------------------------------------
def conv_kernel_id(g: ConvGeom, n, h, w, op, strides=None, copies: bool = False):
    """(selector, splits) of the igemm kernel that runs this conv product (copies: called with
    the operand copies of the _x forms — F32X3 term images, bf16 copies)."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    d = _desc(g, n, h, w, tuple(strides))[0]
    kid, sp = ctypes.c_int(0), ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv2d_kernel_id_x(ctypes.byref(d), op, 1 if copies else 0, ctypes.byref(kid),
                                                 ctypes.byref(sp)), "conv2d_kernel_id")
    return kid.value, sp.value


def conv_copy_operand_only(g: ConvGeom, n, h, w, op, strides=None) -> bool:
    """True when this conv product (aligned operands) runs on a kernel that reads only the
    operand copies of the _x forms, so its fp32 operand need not be written
    (adaptseg_conv2d_copy_operand_only: the plan the entry points check against)."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    d = _desc(g, n, h, w, tuple(strides))[0]
    only = ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv2d_copy_operand_only(ctypes.byref(d), op, ctypes.byref(only)),
          "conv2d_copy_operand_only")
    return bool(only.value)


def timing_enable(selector: int = -1, enable: bool = True):
    check(_lib.lib().adaptseg_timing_enable(1 if enable else 0, int(selector)), "timing_enable")


MEM_KERNELS = {1000: "upsample_fwd_kernel", 1001: "upsample_bwd_{x,y}_kernel", 1002: "softmax_fwd",
               1003: "softmax_bwd", 1004: "ce_fwd (+final)", 1005: "ce_bwd", 1006: "bn_apply2d_kernel",
               1007: "bn_bwd_apply2d_kernel", 1008: "up2_relu_cat_fwd_kernel", 1009: "up2_relu_cat_bwd_kernel",
               1010: "grid_warp_fwd_kernel", 1011: "grid_warp_dflow_kernel",
               1012: "grid_warp input-gradient scatter (memset + absmax + scatter + convert)",
               1013: "bn_reduce_kernel<0> (stats)", 1014: "bn_reduce_kernel<1> (backward sums)",
               1015: "splitk_reduce{4}_kernel"}


def timing_reserve(pairs: int):
    """Create ``pairs`` timing event pairs now (outside the timed region)."""
    check(_lib.lib().adaptseg_timing_reserve(int(pairs)), "timing_reserve")


def timing_enable_mem(enable: bool = True):
    """Record every HBM-bound interp / loss / BN-apply launch with its algorithmic bytes."""
    check(_lib.lib().adaptseg_timing_enable_mem(1 if enable else 0), "timing_enable_mem")


def timing_read_id(kernel_id: int):
    """(total_ms, total_units, launches) of the recorded launches of one kernel id (conv GEMMs:
    the kernels' execution time, hipExtLaunchKernel events)."""
    ms, un, n = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0)
    check(_lib.lib().adaptseg_timing_read_id(int(kernel_id), ctypes.byref(ms), ctypes.byref(un),
                                             ctypes.byref(n)), "timing_read_id")
    return ms.value, un.value, n.value


def timing_enable_stream(enable: bool = True):
    """Conv GEMMs: record stream-time event pairs beside the execution-time ones."""
    check(_lib.lib().adaptseg_timing_enable_stream(1 if enable else 0), "timing_enable_stream")


def timing_read_id_stream(kernel_id: int):
    """(total_ms, launches) of the stream-time pairs of one conv kernel id."""
    ms, n = ctypes.c_double(0), ctypes.c_int64(0)
    check(_lib.lib().adaptseg_timing_read_id_stream(int(kernel_id), ctypes.byref(ms), ctypes.byref(n)),
          "timing_read_id_stream")
    return ms.value, n.value


def timing_read():
    """(total_ms, total_flops, launches) of the timed launches since timing_enable()."""
    ms, fl, n = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0)
    check(_lib.lib().adaptseg_timing_read(ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n)),
          "timing_read")
    return ms.value, fl.value, n.value
