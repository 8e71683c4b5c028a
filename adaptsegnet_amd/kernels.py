"""Tensor-level wrappers over the C ABI (include/adaptseg.h).

Activations handed to these functions are contiguous NHWC fp32 CUDA tensors of shape
``[n, h, w, c]`` (the physical layout of a channels_last NCHW tensor) unless a function
says otherwise.  Every call is asynchronous on the current HIP stream; none synchronises.
These are the only functions that launch compute on the hot path — there is no CPU or
eager-PyTorch fallback, and a missing ``libadaptseg.so`` raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import (CONV_BWD_DATA, CONV_BWD_WEIGHT, CONV_FWD, EPI_ACCUMULATE, EPI_LEAKY,
                   EPI_LEAKY_GRAD, EPI_RELU, EPI_RELU_GRAD, EPI_RESIDUAL, MATH_BF16, MATH_BF16_WIDE, MATH_F32,
                   ConvDesc, check)

__all__ = [
    "ConvGeom", "set_conv_math", "get_conv_math", "MATH_F32", "MATH_BF16", "MATH_BF16_WIDE", "conv_fwd", "conv_fwd_bnstats", "conv_dgrad_bnsums", "bn_bwd_tiles", "conv_dgrad", "conv_wgrad", "bn_fwd_train",
    "bn_fwd_train_tiles", "bn_fwd_infer", "bn_bwd",
    "maxpool_fwd", "maxpool_bwd", "upsample_fwd", "upsample_bwd", "softmax_fwd", "softmax_bwd",
    "ce_fwd", "ce_bwd", "adv_fwd", "adv_bwd", "sgd_step", "adam_step", "zero_", "to_nhwc",
    "axpy", "add_i64", "EPI_ACCUMULATE", "EPI_LEAKY", "EPI_LEAKY_GRAD", "EPI_RELU", "EPI_RELU_GRAD", "EPI_RESIDUAL",
]


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _require(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: expected a CUDA (HIP) tensor, got device {t.device}")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{what}: expected float32, got {t.dtype}")


# ---------------------------------------------------------------------------------------
# Workspace: one growing scratch buffer per (device, stream).  Ops on one stream run in
# order, so reusing it across consecutive calls is race-free.
# ---------------------------------------------------------------------------------------
_WS: dict = {}


def workspace(nbytes: int, device: torch.device) -> torch.Tensor | None:
    if nbytes == 0:
        return None
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        cap = max(nbytes, 0 if buf is None else int(buf.numel() * 1.25))
        buf = torch.empty(cap, dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def _ws_args(nbytes: int, device):
    w = workspace(nbytes, device)
    return (ctypes.c_void_p(w.data_ptr()) if w is not None else None), ctypes.c_size_t(nbytes)


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


_DESC_CACHE: dict = {}
_CONV_MATH = [MATH_F32]


def set_conv_math(math: int) -> None:
    """Process-wide conv arithmetic: MATH_F32 (fp32 MFMA, default) or MATH_BF16 (operands
    rounded to bf16, fp32 accumulate: BASELINE config c5).  Workspace sizes depend on it,
    so the descriptor cache is keyed on it."""
    check(_lib.lib().adaptseg_conv_set_math(int(math)), "conv_set_math")
    _CONV_MATH[0] = int(math)


def get_conv_math() -> int:
    m = ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv_get_math(ctypes.byref(m)), "conv_get_math")
    return m.value


def _desc(g: ConvGeom, n, h, w, strides):
    key = (g, n, h, w, strides, _CONV_MATH[0])
    d = _DESC_CACHE.get(key)
    if d is None:
        oh, ow = g.out_hw(h, w)
        d = ConvDesc()
        d.n, d.c, d.h, d.w = n, g.cin, h, w
        for i in range(4):
            d.in_stride[i] = strides[i]
        d.k, d.oh, d.ow = g.cout, oh, ow
        d.kh, d.kw, d.stride, d.nseg = g.kh, g.kw, g.stride, g.nseg
        for i in range(g.nseg):
            d.pad[i] = g.pads[i]
            d.dil[i] = g.dils[i]
        ws = {}
        for op in (CONV_FWD, CONV_BWD_DATA, CONV_BWD_WEIGHT):
            b = ctypes.c_size_t(0)
            check(_lib.lib().adaptseg_conv2d_workspace_size(ctypes.byref(d), op, ctypes.byref(b)),
                  "conv2d_workspace_size")
            ws[op] = b.value
        d = (d, ws, oh, ow)
        _DESC_CACHE[key] = d
    return d


def nhwc_strides(n, h, w, c):
    """(n, c, h, w) element strides of a contiguous NHWC buffer."""
    return (h * w * c, 1, w * c, c)


def _ptrs(ts):
    return _lib.ptr_array([None if t is None else t.data_ptr() for t in ts])


def conv_fwd(g: ConvGeom, x: torch.Tensor, n: int, h: int, w: int, weights, biases=None,
             strides=None, out=None, res=None, flags: int = 0) -> torch.Tensor:
    """y[n,oh,ow,cout] = sum_seg conv(x, w_seg) + sum_seg b_seg (+res) (EPI_LEAKY / EPI_RELU)."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    d, ws, oh, ow = _desc(g, n, h, w, tuple(strides))
    if out is None:
        out = torch.empty((n, oh, ow, g.cout), device=x.device, dtype=torch.float32)
    if res is not None:
        flags |= EPI_RESIDUAL
    wp, wsz = _ws_args(ws[CONV_FWD], x.device)
    check(_lib.lib().adaptseg_conv2d_fwd(
        ctypes.byref(d), _p(x), _ptrs(weights), _ptrs(biases) if biases is not None else None,
        _p(res), _p(out), flags, wp, wsz, _stream()), "conv2d_fwd")
    return out


def conv_fwd_bnstats(g: ConvGeom, x: torch.Tensor, n: int, h: int, w: int, weights, strides=None):
    """y = conv(x, w) plus the per-row-tile BatchNorm statistics of y when the kernel can
    produce them: returns (y, (stats, ntiles)) or (y, None)."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    d, ws, oh, ow = _desc(g, n, h, w, tuple(strides))
    out = torch.empty((n, oh, ow, g.cout), device=x.device, dtype=torch.float32)
    sb = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_conv2d_bnstats_size(ctypes.byref(d), ctypes.byref(sb)), "conv2d_bnstats_size")
    stats = torch.empty(sb.value // 4, device=x.device, dtype=torch.float32)
    nt = ctypes.c_int(0)
    wp, wsz = _ws_args(ws[CONV_FWD], x.device)
    check(_lib.lib().adaptseg_conv2d_fwd_bnstats(
        ctypes.byref(d), _p(x), _ptrs(weights), _p(out), _p(stats), sb, ctypes.byref(nt), wp, wsz,
        _stream()), "conv2d_fwd_bnstats")
    return out, ((stats, nt.value) if nt.value > 0 else None)


def conv_dgrad(g: ConvGeom, dy: torch.Tensor, n: int, h: int, w: int, weights, out=None,
               res=None, aux=None, flags: int = 0) -> torch.Tensor:
    """dx[n,h,w,cin] (+)= conv_transpose(dy, w) (+res) (*leaky'(aux), or relu'(aux) with EPI_RELU_GRAD)."""
    d, ws, oh, ow = _desc(g, n, h, w, nhwc_strides(n, h, w, g.cin))
    if out is None:
        out = torch.empty((n, h, w, g.cin), device=dy.device, dtype=torch.float32)
    if res is not None:
        flags |= EPI_RESIDUAL
    if aux is not None and not flags & EPI_RELU_GRAD:
        flags |= EPI_LEAKY_GRAD
    wp, wsz = _ws_args(ws[CONV_BWD_DATA], dy.device)
    check(_lib.lib().adaptseg_conv2d_bwd_data(
        ctypes.byref(d), _p(dy), _ptrs(weights), _p(res), _p(aux), _p(out), flags, wp, wsz,
        _stream()), "conv2d_bwd_data")
    return out


def conv_dgrad_bnsums(g: ConvGeom, dy: torch.Tensor, n: int, h: int, w: int, weights, bn_x, mean,
                      invstd, bn_weight, bn_bias):
    """dx = conv_transpose(dy, w) plus, when the kernel can fuse them, the row-tile sums of the
    train-mode BN+ReLU backward whose output dx is the gradient of (bn_x: that BN's input):
    returns (dx, (partial, ntiles)) or (dx, None)."""
    d, ws, oh, ow = _desc(g, n, h, w, nhwc_strides(n, h, w, g.cin))
    dx = torch.empty((n, h, w, g.cin), device=dy.device, dtype=torch.float32)
    sb = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_conv2d_bnsums_size(ctypes.byref(d), ctypes.byref(sb)), "conv2d_bnsums_size")
    partial = torch.empty(sb.value // 4, device=dy.device, dtype=torch.float32)
    nt = ctypes.c_int(0)
    wp, wsz = _ws_args(ws[CONV_BWD_DATA], dy.device)
    check(_lib.lib().adaptseg_conv2d_bwd_data_bnsums(
        ctypes.byref(d), _p(dy), _ptrs(weights), _p(dx), _p(bn_x), _p(mean), _p(invstd), _p(bn_weight),
        _p(bn_bias), _p(partial), sb, ctypes.byref(nt), wp, wsz, _stream()), "conv2d_bwd_data_bnsums")
    return dx, ((partial, nt.value) if nt.value > 0 else None)


def conv_wgrad(g: ConvGeom, dy: torch.Tensor, x: torch.Tensor, n: int, h: int, w: int, dws,
               dbs=None, strides=None, accumulate: bool = True) -> None:
    """dw_seg (+)= sum dy (x) x_gathered ; db_seg (+)= sum dy."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    d, ws, oh, ow = _desc(g, n, h, w, tuple(strides))
    wp, wsz = _ws_args(ws[CONV_BWD_WEIGHT], dy.device)
    check(_lib.lib().adaptseg_conv2d_bwd_weight(
        ctypes.byref(d), _p(dy), _p(x), _ptrs(dws), _ptrs(dbs) if dbs is not None else None,
        EPI_ACCUMULATE if accumulate else 0, wp, wsz, _stream()), "conv2d_bwd_weight")


# ---------------------------------------------------------------------------------------
# BatchNorm (x as [rows, C])
# ---------------------------------------------------------------------------------------
_BN_WS: dict = {}


def _bn_ws(rows, c):
    key = (rows, c)
    v = _BN_WS.get(key)
    if v is None:
        b = ctypes.c_size_t(0)
        check(_lib.lib().adaptseg_bn_workspace_size(rows, c, ctypes.byref(b)), "bn_workspace_size")
        v = _BN_WS[key] = b.value
    return v


def bn_fwd_train(x, weight, bias, running_mean, running_var, momentum, eps, res=None,
                 relu=True, out=None):
    rows, c = x.numel() // x.shape[-1], x.shape[-1]
    y = torch.empty_like(x) if out is None else out
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    invstd = torch.empty(c, device=x.device, dtype=torch.float32)
    wp, wsz = _ws_args(_bn_ws(rows, c), x.device)
    check(_lib.lib().adaptseg_bn_fwd_train(
        rows, c, _p(x), _p(weight), _p(bias), _p(running_mean), _p(running_var),
        float(momentum), float(eps), _p(mean), _p(invstd), _p(res), _p(y), int(relu),
        wp, wsz, _stream()), "bn_fwd_train")
    return y, mean, invstd


def bn_fwd_train_tiles(x, tiles, weight, bias, running_mean, running_var, momentum, eps, res=None,
                       relu=True, out=None):
    """bn_fwd_train whose statistics come from conv_fwd_bnstats's row tiles."""
    stats, ntiles = tiles
    rows, c = x.numel() // x.shape[-1], x.shape[-1]
    y = torch.empty_like(x) if out is None else out
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    invstd = torch.empty(c, device=x.device, dtype=torch.float32)
    check(_lib.lib().adaptseg_bn_fwd_train_tiles(
        rows, c, _p(stats), int(ntiles), _p(x), _p(weight), _p(bias), _p(running_mean),
        _p(running_var), float(momentum), float(eps), _p(mean), _p(invstd), _p(res), _p(y),
        int(relu), _stream()), "bn_fwd_train_tiles")
    return y, mean, invstd


def bn_fwd_infer(x, weight, bias, running_mean, running_var, eps, res=None, relu=True, out=None):
    rows, c = x.numel() // x.shape[-1], x.shape[-1]
    y = torch.empty_like(x) if out is None else out
    check(_lib.lib().adaptseg_bn_fwd_infer(
        rows, c, _p(x), _p(weight), _p(bias), _p(running_mean), _p(running_var), float(eps),
        _p(res), _p(y), int(relu), _stream()), "bn_fwd_infer")
    return y


def bn_bwd(dy, y, x, weight, mean, invstd, relu=True, dx=None, dres=None, train=True, bias=None):
    """dx = BN-backward(g), g = dy*[y>0] if relu; dres receives g.  dx/dres may alias dy.
    y=None with relu (train mode): the mask is recomputed from x, weight and bias."""
    rows, c = dy.numel() // dy.shape[-1], dy.shape[-1]
    if dx is None:
        dx = torch.empty_like(dy)
    wp, wsz = _ws_args(_bn_ws(rows, c) if train else 0, dy.device)
    check(_lib.lib().adaptseg_bn_bwd(
        rows, c, _p(dy), _p(y), _p(x), _p(weight), _p(bias), _p(mean), _p(invstd), _p(dx),
        _p(dres), int(relu), 1 if train else 0, wp, wsz, _stream()), "bn_bwd")
    return dx


def bn_bwd_tiles(dy, x, weight, bias, mean, invstd, sums, dx=None, dres=None):
    """Train-mode BN+ReLU backward (mask recomputed from x) from the row-tile sums that
    conv_dgrad_bnsums fused into the data-gradient epilogue.  dx may alias dy."""
    partial, nt = sums
    rows, c = dy.numel() // dy.shape[-1], dy.shape[-1]
    if dx is None:
        dx = torch.empty_like(dy)
    coef = torch.empty(2 * c, device=dy.device, dtype=torch.float32)
    check(_lib.lib().adaptseg_bn_bwd_tiles(
        rows, c, _p(partial), nt, _p(dy), _p(x), _p(weight), _p(bias), _p(mean), _p(invstd), _p(coef),
        _p(dx), _p(dres), _stream()), "bn_bwd_tiles")
    return dx


ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2   # the BN entry points' activation codes


def bn_bwd_affine(dy, y, x, weight, bias, mean, invstd, act, dweight=None, dbias=None, dx=None):
    """Train-mode BN backward with trainable affine parameters: dx, plus dweight/dbias
    accumulated (sum g*xhat, sum g).  act: ACT_NONE / ACT_RELU / ACT_LEAKY (mask from y, or
    from x when y is None).  dx may alias dy."""
    rows, c = dy.numel() // dy.shape[-1], dy.shape[-1]
    if dx is None:
        dx = torch.empty_like(dy)
    wp, wsz = _ws_args(_bn_ws(rows, c), dy.device)
    check(_lib.lib().adaptseg_bn_bwd_affine(
        rows, c, _p(dy), _p(y), _p(x), _p(weight), _p(bias), _p(mean), _p(invstd), _p(dx), None,
        int(act), _p(dweight), _p(dbias), wp, wsz, _stream()), "bn_bwd_affine")
    return dx


# ---------------------------------------------------------------------------------------
# Warper: decoder input (ReLU + x2 upsample + skip concat) and the prediction warp
# ---------------------------------------------------------------------------------------
def up2_relu_cat_fwd(s, d):
    """NHWC up2(relu(cat(s, d))) at twice the resolution; s may be None."""
    n, h, w, cd = d.shape
    cs = 0 if s is None else s.shape[-1]
    out = torch.empty((n, 2 * h, 2 * w, cs + cd), device=d.device, dtype=torch.float32)
    check(_lib.lib().adaptseg_up2_relu_cat_fwd(n, h, w, cs, cd, _p(s), _p(d), _p(out), _stream()),
          "up2_relu_cat_fwd")
    return out


def up2_relu_cat_bwd(s, d, dout, ds=None, dd=None):
    """(ds, dd) = masked split of up2^T(dout); ds is None when s is None."""
    n, h, w, cd = d.shape
    cs = 0 if s is None else s.shape[-1]
    if dd is None:
        dd = torch.empty_like(d)
    if s is not None and ds is None:
        ds = torch.empty_like(s)
    check(_lib.lib().adaptseg_up2_relu_cat_bwd(n, h, w, cs, cd, _p(s), _p(d), _p(dout), _p(ds), _p(dd),
                                               _stream()), "up2_relu_cat_bwd")
    return ds, dd


def grid_warp_fwd(flow, x1, x2):
    """ResNetMulti.warp of both heads (NHWC [n,h,w,c]; x1 may be None) by one NHWC warp field."""
    n, h, w, c = x2.shape
    fc = flow.shape[-1]
    y1 = None if x1 is None else torch.empty_like(x1)
    y2 = torch.empty_like(x2)
    check(_lib.lib().adaptseg_grid_warp_fwd(n, c, h, w, fc, _p(flow), _p(x1), _p(x2), _p(y1), _p(y2),
                                            _stream()), "grid_warp_fwd")
    return y1, y2


def grid_warp_bwd(flow, x1, x2, dy1, dy2, need_dflow=True, need_dx1=True, need_dx2=True):
    """-> (dflow, dx1, dx2); entries not requested (or without their dy) are None."""
    ref = dy2 if dy2 is not None else dy1
    n, h, w, c = ref.shape
    fc = flow.shape[-1]
    dflow = torch.empty_like(flow) if need_dflow else None
    dx1 = torch.empty_like(dy1) if (need_dx1 and dy1 is not None) else None
    dx2 = torch.empty_like(dy2) if (need_dx2 and dy2 is not None) else None
    nbytes = 0
    if dx1 is not None or dx2 is not None:
        b = ctypes.c_size_t(0)
        check(_lib.lib().adaptseg_grid_warp_bwd_workspace_size(n, c, h, w, ctypes.byref(b)),
              "grid_warp_bwd_workspace_size")
        nbytes = b.value
    wp, wsz = _ws_args(nbytes, ref.device)
    check(_lib.lib().adaptseg_grid_warp_bwd(
        n, c, h, w, fc, _p(flow), _p(x1 if dy1 is not None else None), _p(x2 if dy2 is not None else None),
        _p(dy1), _p(dy2), _p(dflow), _p(dx1), _p(dx2), wp, wsz, _stream()), "grid_warp_bwd")
    return dflow, dx1, dx2


# ---------------------------------------------------------------------------------------
# Pooling / interpolation / softmax / losses
# ---------------------------------------------------------------------------------------
def maxpool_fwd(x, k=3, s=2, p=1):
    n, h, w, c = x.shape
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    y = torch.empty((n, oh, ow, c), device=x.device, dtype=torch.float32)
    am = torch.empty((n, oh, ow, c), device=x.device, dtype=torch.uint8)
    check(_lib.lib().adaptseg_maxpool2d_fwd(n, c, h, w, oh, ow, k, s, p, _p(x), _p(y), _p(am),
                                            _stream()), "maxpool2d_fwd")
    return y, am


def maxpool_bwd(dy, am, h, w, k=3, s=2, p=1):
    n, oh, ow, c = dy.shape
    dx = torch.empty((n, h, w, c), device=dy.device, dtype=torch.float32)
    check(_lib.lib().adaptseg_maxpool2d_bwd(n, c, h, w, oh, ow, k, s, p, _p(dy), _p(am), _p(dx),
                                            _stream()), "maxpool2d_bwd")
    return dx


def upsample_fwd(x, oh, ow):
    n, h, w, c = x.shape
    y = torch.empty((n, oh, ow, c), device=x.device, dtype=torch.float32)
    check(_lib.lib().adaptseg_upsample_bilinear_fwd(n, c, h, w, oh, ow, _p(x), _p(y), _stream()),
          "upsample_bilinear_fwd")
    return y


def upsample_bwd(dy, h, w, out=None, accumulate=False):
    n, oh, ow, c = dy.shape
    if out is None:
        out = torch.empty((n, h, w, c), device=dy.device, dtype=torch.float32)
    nbytes = n * oh * w * c * 4
    wp, wsz = _ws_args(nbytes, dy.device)
    check(_lib.lib().adaptseg_upsample_bilinear_bwd(
        n, c, h, w, oh, ow, _p(dy), _p(out), EPI_ACCUMULATE if accumulate else 0, wp, wsz,
        _stream()), "upsample_bilinear_bwd")
    return out


def softmax_fwd(x):
    c = x.shape[-1]
    y = torch.empty_like(x)
    check(_lib.lib().adaptseg_softmax_fwd(x.numel() // c, c, _p(x), _p(y), _stream()),
          "softmax_fwd")
    return y


def softmax_bwd(y, dy, out=None, accumulate=False):
    c = y.shape[-1]
    if out is None:
        out = torch.empty_like(y)
    check(_lib.lib().adaptseg_softmax_bwd(y.numel() // c, c, _p(y), _p(dy), _p(out),
                                          EPI_ACCUMULATE if accumulate else 0, _stream()),
          "softmax_bwd")
    return out


def ce_fwd(logits, labels, ignore=255, class_weight=None):
    """Returns a 2-element device tensor [loss, denominator]."""
    c = logits.shape[-1]
    rows = logits.numel() // c
    out = torch.empty(2, device=logits.device, dtype=torch.float32)
    b = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_ce_workspace_size(rows, ctypes.byref(b)), "ce_workspace_size")
    wp, wsz = _ws_args(b.value, logits.device)
    check(_lib.lib().adaptseg_softmax_ce_fwd(rows, c, _p(logits), _p(labels), int(ignore),
                                             _p(class_weight), _p(out), wp, wsz, _stream()),
          "softmax_ce_fwd")
    return out


def ce_bwd(logits, labels, out2, grad_loss, ignore=255, class_weight=None, dl=None,
           accumulate=False):
    c = logits.shape[-1]
    rows = logits.numel() // c
    if dl is None:
        dl = torch.empty_like(logits)
    check(_lib.lib().adaptseg_softmax_ce_bwd(rows, c, _p(logits), _p(labels), int(ignore),
                                             _p(class_weight), _p(out2), _p(grad_loss), _p(dl),
                                             EPI_ACCUMULATE if accumulate else 0, _stream()),
          "softmax_ce_bwd")
    return dl


def adv_fwd(x, target: float, kind: int):
    n = x.numel()
    loss = torch.empty(1, device=x.device, dtype=torch.float32)
    b = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_adv_workspace_size(n, ctypes.byref(b)), "adv_workspace_size")
    wp, wsz = _ws_args(b.value, x.device)
    check(_lib.lib().adaptseg_adv_loss_fwd(n, _p(x), float(target), int(kind), _p(loss), wp, wsz,
                                           _stream()), "adv_loss_fwd")
    return loss


def adv_bwd(x, target: float, kind: int, grad_loss, dx=None, accumulate=False):
    if dx is None:
        dx = torch.empty_like(x)
    check(_lib.lib().adaptseg_adv_loss_bwd(x.numel(), _p(x), float(target), int(kind),
                                           _p(grad_loss), _p(dx),
                                           EPI_ACCUMULATE if accumulate else 0, _stream()),
          "adv_loss_bwd")
    return dx


# ---------------------------------------------------------------------------------------
# Optimisers and plumbing
# ---------------------------------------------------------------------------------------
def sgd_step(param, grad, mom, lr, momentum, weight_decay, grad_scale=1.0, multiplicity=1,
             first_step=False):
    check(_lib.lib().adaptseg_sgd_step(param.numel(), _p(param), _p(grad), _p(mom), float(lr),
                                       float(momentum), float(weight_decay), float(grad_scale),
                                       int(multiplicity), 1 if first_step else 0, _stream()),
          "sgd_step")


def adam_step(param, grad, m, v, lr, beta1, beta2, eps, step, grad_scale=1.0):
    check(_lib.lib().adaptseg_adam_step(param.numel(), _p(param), _p(grad), _p(m), _p(v),
                                        float(lr), float(beta1), float(beta2), float(eps),
                                        int(step), float(grad_scale), _stream()), "adam_step")


def zero_(t: torch.Tensor) -> torch.Tensor:
    check(_lib.lib().adaptseg_zero(_p(t), t.numel() * t.element_size(), _stream()), "zero")
    return t


def to_nhwc(t: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor (any strides) -> contiguous NHWC buffer [n, h, w, c]."""
    _require(t, "to_nhwc")
    n, c, h, w = t.shape
    st = (ctypes.c_int64 * 4)(*t.stride())
    out = torch.empty((n, h, w, c), device=t.device, dtype=torch.float32)
    check(_lib.lib().adaptseg_to_nhwc(n, c, h, w, st, _p(t), _p(out), _stream()), "to_nhwc")
    return out


def axpy(alpha, src, dst, accumulate=True):
    check(_lib.lib().adaptseg_axpy(src.numel(), float(alpha), _p(src), _p(dst),
                                   EPI_ACCUMULATE if accumulate else 0, _stream()), "axpy")
    return dst


def add_i64(t: torch.Tensor, v: int = 1):
    check(_lib.lib().adaptseg_add_i64(_p(t), t.numel(), int(v), _stream()), "add_i64")


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
def conv_kernel_id(g: ConvGeom, n, h, w, op, strides=None):
    """(selector, splits) of the igemm kernel that runs this conv product."""
    strides = strides or nhwc_strides(n, h, w, g.cin)
    d = _desc(g, n, h, w, tuple(strides))[0]
    kid, sp = ctypes.c_int(0), ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv2d_kernel_id(ctypes.byref(d), op, ctypes.byref(kid), ctypes.byref(sp)),
          "conv2d_kernel_id")
    return kid.value, sp.value


def timing_enable(selector: int = -1, enable: bool = True):
    check(_lib.lib().adaptseg_timing_enable(1 if enable else 0, int(selector)), "timing_enable")


MEM_KERNELS = {1000: "upsample_fwd_kernel", 1001: "upsample_bwd_{x,y}_kernel", 1002: "softmax_fwd",
               1003: "softmax_bwd", 1004: "ce_fwd (+final)", 1005: "ce_bwd", 1006: "bn_apply2d_kernel",
               1007: "bn_bwd_apply2d_kernel", 1008: "up2_relu_cat_fwd_kernel", 1009: "up2_relu_cat_bwd_kernel",
               1010: "grid_warp_fwd_kernel", 1011: "grid_warp_dflow_kernel",
               1012: "grid_warp input-gradient scatter (memset + absmax + scatter + convert)"}


def timing_enable_mem(enable: bool = True):
    """Record every HBM-bound interp / loss / BN-apply launch with its algorithmic bytes."""
    check(_lib.lib().adaptseg_timing_enable_mem(1 if enable else 0), "timing_enable_mem")


def timing_read_id(kernel_id: int):
    """(total_ms, total_units, launches) of the recorded launches of one kernel id."""
    ms, un, n = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0)
    check(_lib.lib().adaptseg_timing_read_id(int(kernel_id), ctypes.byref(ms), ctypes.byref(un),
                                             ctypes.byref(n)), "timing_read_id")
    return ms.value, un.value, n.value


def timing_read():
    """(total_ms, total_flops, launches) of the timed launches since timing_enable()."""
    ms, fl, n = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int64(0)
    check(_lib.lib().adaptseg_timing_read(ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n)),
          "timing_read")
    return ms.value, fl.value, n.value
