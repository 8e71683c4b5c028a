"""``torch.ops.adaptseg``: the native op surface as PyTorch custom operators.

Every compute launch of the package goes through one of these operators (registered with
``torch.library``: a schema, a CUDA (= HIP on ROCm) kernel and a fake/meta kernel), so the
launches are visible to the dispatcher — torch.profiler records them by name, FakeTensor /
``torch.library.opcheck`` can trace them — while the native boundary stays the C ABI of
include/adaptseg.h: each CUDA kernel below is a thin ctypes call into libadaptseg.so.

There is no CPU kernel: calling an op on CPU tensors raises NotImplementedError from the
dispatcher (the product path has no fallback).  All ops are out-variant: outputs (and
state such as BN running statistics or optimiser buffers) are caller-allocated and declared
mutable (``Tensor(a!)``) in the schema, every op returns ``()``, and ``adaptsegnet_amd.kernels``
allocates and calls them.  Activations are NHWC buffers ``[n, h, w, c]`` (the physical layout
of channels_last NCHW tensors) unless an argument says otherwise; conv weights are any
tensors whose memory is [Cout][KH][KW][Cin] (the modules' NCHW-shaped channels_last
parameters), their logical shape given by ``w_shape`` = [Cout, Cin, KH, KW].  Some engine
calls alias a read-only input with a mutable output (in-place BN backward, residual folded
into the data-gradient output); the kernels support that, and it is why these ops are not
meant for torch.compile's functionalization.

Reference call sites the ops stand in for (file:line in /root/reference):
  conv2d_*            nn.Conv2d in model/deeplab_multi.py:64-75,112,128 / discriminator.py:10-14
                      (conv2d_wpack: the per-step weight pack, optimiser train:532-540 between steps)
  bn_*                nn.BatchNorm2d (+ReLU, residual)  model/deeplab_multi.py:65-101,130-135
  maxpool2d_*         nn.MaxPool2d(3, 2, 1)             model/deeplab_multi.py:135
  upsample_bilinear_* nn.Upsample(bilinear, align_corners=True)  model/deeplab_multi.py:188-189
  softmax_*           F.softmax(pred)                   train_gta2cityscapes_multi.py:617-618
  softmax_ce_*        nn.CrossEntropyLoss(ignore_index=255) / CrossEntropy2d  train:546, utils/loss.py:7-36
  adv_loss_*          BCEWithLogitsLoss / MSELoss vs a constant label  train:542-545,620-624
  sgd_step/adam_step  optim.SGD / optim.Adam            train:532-540
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import CONV_BWD_DATA, CONV_BWD_WEIGHT, CONV_FWD, MATH_F32X3, ConvDesc, check

LIB = torch.library.Library("adaptseg", "DEF")


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _pf(t, n, what):
    """fp32 operand pointer, checked on the host before any launch: float32 and exactly ``n``
    elements (a tensor of the wrong dtype or size must raise here, not fault on the GPU)."""
    if t is None:
        return None
    if t.dtype != torch.float32 or t.numel() != n:
        raise RuntimeError(f"{what}: expected a float32 tensor of {n} elements, got {t.dtype} {tuple(t.shape)}")
    return ctypes.c_void_p(t.data_ptr())


def _pc(t, n, what):
    """Operand-copy pointer (bf16 image of n elements, or the 3n of F32X3 term images)."""
    if t is None:
        return None
    if t.dtype != torch.bfloat16 or t.numel() not in (n, 3 * n):
        raise RuntimeError(f"{what}: expected a bf16 copy of {n} (or 3 x {n}) elements, got {t.dtype} "
                           f"{tuple(t.shape)}")
    return ctypes.c_void_p(t.data_ptr())


def _pfb(t, n, what):
    """(fp32 pointer, bf16 pointer) of a tensor of n elements stored as either."""
    if t is None:
        return None, None
    if t.dtype == torch.bfloat16:
        return None, _pc(t, n, what)
    return _pf(t, n, what), None


def _pbits(t, n, what):
    """Mask-bitmap pointer: int32 words, one bit per element of an n-element tensor."""
    if t is None:
        return None
    if t.dtype != torch.int32 or t.numel() * 32 != n:
        raise RuntimeError(f"{what}: expected an int32 bitmap of {n // 32} words, got {t.dtype} {tuple(t.shape)}")
    return ctypes.c_void_p(t.data_ptr())


def _ptrs(ts):
    return _lib.ptr_array([None if t is None else t.data_ptr() for t in ts])


# One growing scratch buffer per (device, stream): ops on one stream run in order, so reusing
# it across consecutive calls is race-free.  Caller-owned from the C ABI's point of view.
_WS: dict = {}


def workspace(nbytes: int, device: torch.device):
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
# Conv descriptors (host planning only: no GPU needed)
# ---------------------------------------------------------------------------------------
_DESC_CACHE: dict = {}
_CONV_MATH = [MATH_F32X3]   # the library's default (adaptseg_conv_get_math)
OPT_X3H, OPT_G16_WIDE = 1, 2   # adaptseg_conv_option
_OPTS: dict = {}               # adaptseg_conv_get_option, read on first use (the library reads the environment)


def get_option(opt: int) -> int:
    if opt not in _OPTS:
        m = ctypes.c_int(0)
        check(_lib.lib().adaptseg_conv_get_option(int(opt), ctypes.byref(m)), "conv_get_option")
        _OPTS[opt] = m.value
    return _OPTS[opt]


def set_option(opt: int, value: int) -> None:
    check(_lib.lib().adaptseg_conv_set_option(int(opt), int(value)), "conv_set_option")
    _OPTS[opt] = int(value)


def conv_desc(n, c, h, w, strides, cout, kh, kw, stride, pads, dils):
    """(ConvDesc, {op: workspace bytes}, oh, ow) of one conv product, cached."""
    key = (n, c, h, w, strides, cout, kh, kw, stride, pads, dils, _CONV_MATH[0], get_option(OPT_X3H),
           get_option(OPT_G16_WIDE))
    d = _DESC_CACHE.get(key)
    if d is None:
        p, dl = pads[0], dils[0]
        oh = (h + 2 * p - dl * (kh - 1) - 1) // stride + 1
        ow = (w + 2 * p - dl * (kw - 1) - 1) // stride + 1
        desc = ConvDesc()
        desc.n, desc.c, desc.h, desc.w = n, c, h, w
        for i in range(4):
            desc.in_stride[i] = strides[i]
        desc.k, desc.oh, desc.ow = cout, oh, ow
        desc.kh, desc.kw, desc.stride, desc.nseg = kh, kw, stride, len(pads)
        for i in range(len(pads)):
            desc.pad[i] = pads[i]
            desc.dil[i] = dils[i]
        ws = {}
        for op in (CONV_FWD, CONV_BWD_DATA, CONV_BWD_WEIGHT):
            b = ctypes.c_size_t(0)
            check(_lib.lib().adaptseg_conv2d_workspace_size(ctypes.byref(desc), op, ctypes.byref(b)),
                  "conv2d_workspace_size")
            ws[op] = b.value
        d = _DESC_CACHE[key] = (desc, ws, oh, ow)
    return d


def set_math(math: int) -> None:
    check(_lib.lib().adaptseg_conv_set_math(int(math)), "conv_set_math")
    _CONV_MATH[0] = int(math)


def _wdesc(in_shape, in_stride, w_shape, stride, pad, dil):
    co, _ci, kh, kw = w_shape
    n, c, h, w = in_shape
    return conv_desc(n, c, h, w, tuple(in_stride), co, kh, kw, stride, tuple(pad), tuple(dil))


def _prod(shape):
    out = 1
    for v in shape:
        out *= int(v)
    return out


def _nhwc_strides(n, h, w, c):
    return (h * w * c, 1, w * c, c)


# ---------------------------------------------------------------------------------------
# Registration
# ---------------------------------------------------------------------------------------
def _fake(*args, **kwargs):
    return None


NAMES: list = []


def _op(schema):
    """Define adaptseg::<schema> with the decorated function as its CUDA kernel."""
    name = schema.split("(", 1)[0]

    def deco(fn):
        NAMES.append(name)
        LIB.define(schema)
        LIB.impl(name, fn, "CUDA")
        torch.library.register_fake(f"adaptseg::{name}", _fake, lib=LIB)
        return fn
    return deco


# ---- convolution ------------------------------------------------------------------------
@_op("conv2d_wpack(Tensor[] weight, Tensor(a!) pack, int[] in_shape, int[] in_stride, int[] w_shape, int stride, "
     "int[] pad, int[] dil, int op) -> ()")
def _conv2d_wpack(weight, pack, in_shape, in_stride, w_shape, stride, pad, dil, op):
    d, _, _, _ = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)
    check(_lib.lib().adaptseg_conv2d_wpack(ctypes.byref(d), int(op), _ptrs(weight), _p(pack), pack.numel(),
                                           _stream()), "conv2d_wpack")


@_op("conv2d_fwd(Tensor? x, Tensor? xb, Tensor[] weight, Tensor? wpack, Tensor?[] bias, Tensor? res, "
     "Tensor(a!)? out, Tensor(b!)? outb, int[] in_shape, int[] in_stride, int[] w_shape, int stride, int[] pad, "
     "int[] dil, int flags) -> ()")
def _conv2d_fwd(x, xb, weight, wpack, bias, res, out, outb, in_shape, in_stride, w_shape, stride, pad, dil, flags):
    d, ws, oh, ow = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)
    wp, wsz = _ws_args(ws[CONV_FWD], (out if out is not None else outb).device)
    nx, ny = _prod(in_shape), in_shape[0] * oh * ow * w_shape[0]
    check(_lib.lib().adaptseg_conv2d_fwd_x(
        ctypes.byref(d), _pf(x, nx, "conv2d_fwd x"), _pc(xb, nx, "conv2d_fwd xb"), _ptrs(weight), _p(wpack),
        _ptrs(bias) if len(bias) else None, _pf(res, ny, "conv2d_fwd res"),
        _pf(out, ny, "conv2d_fwd out"), _pc(outb, ny, "conv2d_fwd outb"), flags, wp, wsz, _stream()), "conv2d_fwd")


@_op("conv2d_fwd_bnstats(Tensor? x, Tensor? xb, Tensor[] weight, Tensor? wpack, Tensor(a!)? out, Tensor(c!)? outb, "
     "Tensor(b!) stats, int[] in_shape, int[] in_stride, int[] w_shape, int stride, int[] pad, int[] dil, "
     "int ntiles) -> ()")
def _conv2d_fwd_bnstats(x, xb, weight, wpack, out, outb, stats, in_shape, in_stride, w_shape, stride, pad, dil,
                        ntiles):
    d, ws, oh, ow = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)
    wp, wsz = _ws_args(ws[CONV_FWD], stats.device)
    nt = ctypes.c_int(0)
    nx, ny = _prod(in_shape), in_shape[0] * oh * ow * w_shape[0]
    check(_lib.lib().adaptseg_conv2d_fwd_bnstats_x(
        ctypes.byref(d), _pf(x, nx, "conv2d_fwd_bnstats x"), _pc(xb, nx, "conv2d_fwd_bnstats xb"), _ptrs(weight),
        _p(wpack), _pf(out, ny, "conv2d_fwd_bnstats out"), _pc(outb, ny, "conv2d_fwd_bnstats outb"), _p(stats),
        ctypes.c_size_t(stats.numel() * 4), ctypes.byref(nt), wp, wsz, _stream()), "conv2d_fwd_bnstats")
    if nt.value != ntiles:
        raise RuntimeError(f"conv2d_fwd_bnstats: planned {ntiles} statistics tiles, the launch produced "
                           f"{nt.value} (unaligned operand?)")


def _abn(mean, invstd, bnw, bnb):
    return _lib.OperandBN(mean.data_ptr(), invstd.data_ptr(), None if bnw is None else bnw.data_ptr(),
                          None if bnb is None else bnb.data_ptr())


_ABN_OK: dict = {}


def operand_bn_ok(in_shape, in_stride, w_shape, stride, pad, dil, op) -> bool:
    """adaptseg_conv2d_operand_bn_ok, cached per product (host planning, no GPU)."""
    key = (tuple(in_shape), tuple(in_stride), tuple(w_shape), stride, tuple(pad), tuple(dil), op, _CONV_MATH[0],
           get_option(OPT_X3H), get_option(OPT_G16_WIDE))
    v = _ABN_OK.get(key)
    if v is None:
        d = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)[0]
        ok = ctypes.c_int(0)
        check(_lib.lib().adaptseg_conv2d_operand_bn_ok(ctypes.byref(d), int(op), ctypes.byref(ok)), "operand_bn_ok")
        v = _ABN_OK[key] = bool(ok.value)
    return v


@_op("conv2d_fwd_bnstats_abn(Tensor x_pre, Tensor mean, Tensor invstd, Tensor? bnw, Tensor? bnb, Tensor[] weight, "
     "Tensor? wpack, Tensor(a!) out, Tensor(b!) stats, int[] in_shape, int[] in_stride, int[] w_shape, int stride, "
     "int[] pad, int[] dil, int ntiles) -> ()")
def _conv2d_fwd_bnstats_abn(x_pre, mean, invstd, bnw, bnb, weight, wpack, out, stats, in_shape, in_stride, w_shape,
                            stride, pad, dil, ntiles):
    """conv2d_fwd_bnstats on relu(bn(x_pre)) — the operand BN folded into the gather
    (adaptseg_conv2d_fwd_bnstats_abn)."""
    d, ws, oh, ow = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)
    wp, wsz = _ws_args(ws[CONV_FWD], stats.device)
    nt = ctypes.c_int(0)
    nx, ny = _prod(in_shape), in_shape[0] * oh * ow * w_shape[0]
    a = _abn(mean, invstd, bnw, bnb)
    check(_lib.lib().adaptseg_conv2d_fwd_bnstats_abn(
        ctypes.byref(d), _pf(x_pre, nx, "conv2d_fwd_bnstats_abn x_pre"), ctypes.byref(a), _ptrs(weight), _p(wpack),
        _pf(out, ny, "conv2d_fwd_bnstats_abn out"), _p(stats), ctypes.c_size_t(stats.numel() * 4), ctypes.byref(nt),
        wp, wsz, _stream()), "conv2d_fwd_bnstats_abn")
    if nt.value != ntiles:
        raise RuntimeError(f"conv2d_fwd_bnstats_abn: planned {ntiles} statistics tiles, the launch produced "
                           f"{nt.value} (unaligned operand?)")


@_op("conv2d_bwd_weight_abn(Tensor dy, Tensor x_pre, Tensor mean, Tensor invstd, Tensor? bnw, Tensor? bnb, "
     "Tensor(a!)[] dw, int[] in_shape, int[] in_stride, int[] w_shape, int stride, int[] pad, int[] dil, "
     "int flags) -> ()")
def _conv2d_bwd_weight_abn(dy, x_pre, mean, invstd, bnw, bnb, dw, in_shape, in_stride, w_shape, stride, pad, dil,
                           flags):
    """conv2d_bwd_weight with the x operand relu(bn(x_pre)) (adaptseg_conv2d_bwd_weight_abn)."""
    d, ws, oh, ow = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)
    wp, wsz = _ws_args(ws[CONV_BWD_WEIGHT], dw[0].device)
    nx, ny = _prod(in_shape), in_shape[0] * oh * ow * w_shape[0]
    a = _abn(mean, invstd, bnw, bnb)
    check(_lib.lib().adaptseg_conv2d_bwd_weight_abn(
        ctypes.byref(d), _pf(dy, ny, "conv2d_bwd_weight_abn dy"), _pf(x_pre, nx, "conv2d_bwd_weight_abn x_pre"),
        ctypes.byref(a), _ptrs(dw), flags, wp, wsz, _stream()), "conv2d_bwd_weight_abn")


@_op("bn_fwd_train_tiles_stats(Tensor stats, int ntiles, int rows, int c, Tensor(a!)? running_mean, "
     "Tensor(b!)? running_var, Tensor(d!) mean, Tensor(e!) invstd, float momentum, float eps) -> ()")
def _bn_fwd_train_tiles_stats(stats, ntiles, rows, c, running_mean, running_var, mean, invstd, momentum, eps):
    check(_lib.lib().adaptseg_bn_fwd_train_tiles_stats(
        int(rows), int(c), _p(stats), int(ntiles), _p(running_mean), _p(running_var), float(momentum), float(eps),
        _p(mean), _p(invstd), _stream()), "bn_fwd_train_tiles_stats")


@_op("conv2d_bwd_data(Tensor? dy, Tensor? dyb, Tensor[] weight, Tensor? wpack, Tensor? res, Tensor? resbits, "
     "Tensor? aux, Tensor(a!)? dx, Tensor(b!)? dxb, int[] in_shape, int[] w_shape, int stride, int[] pad, "
     "int[] dil, int flags) -> ()")
def _conv2d_bwd_data(dy, dyb, weight, wpack, res, resbits, aux, dx, dxb, in_shape, w_shape, stride, pad, dil, flags):
    """res: fp32 or bf16, masked by the bitmap resbits (int32 [rows, Cin / 32]) when given; dx None:
    the output is stored in bf16 only (dxb) — bf16 gradient storage (adaptseg_conv2d_bwd_data_xg)."""
    n, c, h, w = in_shape
    d, ws, oh, ow = _wdesc(in_shape, _nhwc_strides(n, h, w, c), w_shape, stride, pad, dil)
    wp, wsz = _ws_args(ws[CONV_BWD_DATA], (dx if dx is not None else dxb).device)
    nx, ny = n * h * w * c, n * oh * ow * w_shape[0]
    check(_lib.lib().adaptseg_conv2d_bwd_data_xg(
        ctypes.byref(d), _pf(dy, ny, "conv2d_bwd_data dy"), _pc(dyb, ny, "conv2d_bwd_data dyb"), _ptrs(weight),
        _p(wpack), *_pfb(res, nx, "conv2d_bwd_data res"), _pbits(resbits, nx, "conv2d_bwd_data resbits"),
        _pf(aux, nx, "conv2d_bwd_data aux"),
        _pf(dx, nx, "conv2d_bwd_data dx"), _pc(dxb, nx, "conv2d_bwd_data dxb"), flags, wp, wsz, _stream()),
        "conv2d_bwd_data")


@_op("conv2d_bwd_data_bnsum(Tensor? dy, Tensor? dyb, Tensor[] weight, Tensor? wpack, Tensor? res, Tensor? resbits, "
     "Tensor(a!)? dx, Tensor(b!)? dxb, int[] in_shape, int[] w_shape, int stride, int[] pad, int[] dil, int flags, "
     "Tensor bnx, Tensor mean, Tensor invstd, Tensor? bnw, Tensor? bnb, Tensor? bits, int mask, Tensor(c!) partial, "
     "int ntiles) -> ()")
def _conv2d_bwd_data_bnsum(dy, dyb, weight, wpack, res, resbits, dx, dxb, in_shape, w_shape, stride, pad, dil, flags,
                           bnx, mean, invstd, bnw, bnb, bits, mask, partial, ntiles):
    """conv2d_bwd_data that also writes the fused BN backward sums of its output (the BN whose
    incoming gradient it is; adaptseg_conv2d_bwd_data_bnsum) into partial [2][Cin][ntiles]."""
    n, c, h, w = in_shape
    d, ws, oh, ow = _wdesc(in_shape, _nhwc_strides(n, h, w, c), w_shape, stride, pad, dil)
    wp, wsz = _ws_args(ws[CONV_BWD_DATA], partial.device)
    nx, ny = n * h * w * c, n * oh * ow * w_shape[0]
    if partial.dtype != torch.float32 or partial.numel() != 2 * c * ntiles:
        raise RuntimeError(f"conv2d_bwd_data_bnsum: partial must be float32 [2][{c}][{ntiles}]")
    bs = _lib.BnSumDesc()
    bs.x, bs.x_bf16 = _pfb(bnx, nx, "conv2d_bwd_data_bnsum bnx")
    bs.mean, bs.invstd, bs.weight, bs.bias = _p(mean), _p(invstd), _p(bnw), _p(bnb)
    bs.bits = _pbits(bits, nx, "conv2d_bwd_data_bnsum bits")
    bs.mask = int(mask)
    bs.partial = _p(partial)
    bs.partial_bytes = partial.numel() * 4
    nt = ctypes.c_int(0)
    check(_lib.lib().adaptseg_conv2d_bwd_data_bnsum(
        ctypes.byref(d), _pf(dy, ny, "conv2d_bwd_data_bnsum dy"), _pc(dyb, ny, "conv2d_bwd_data_bnsum dyb"),
        _ptrs(weight), _p(wpack), *_pfb(res, nx, "conv2d_bwd_data_bnsum res"),
        _pbits(resbits, nx, "conv2d_bwd_data_bnsum resbits"), _pf(dx, nx, "conv2d_bwd_data_bnsum dx"),
        _pc(dxb, nx, "conv2d_bwd_data_bnsum dxb"), flags, ctypes.byref(bs), ctypes.byref(nt), wp, wsz, _stream()),
        "conv2d_bwd_data_bnsum")
    if nt.value != ntiles:
        raise RuntimeError(f"conv2d_bwd_data_bnsum: planned {ntiles} BN-sum tiles, the launch produced {nt.value} "
                           f"(unaligned operand?)")


@_op("conv2d_bwd_weight(Tensor? dy, Tensor? dyb, Tensor? x, Tensor? xb, Tensor(a!)[] dw, Tensor(b!)[] db, "
     "int[] in_shape, int[] in_stride, int[] w_shape, int stride, int[] pad, int[] dil, int flags) -> ()")
def _conv2d_bwd_weight(dy, dyb, x, xb, dw, db, in_shape, in_stride, w_shape, stride, pad, dil, flags):
    d, ws, oh, ow = _wdesc(in_shape, in_stride, w_shape, stride, pad, dil)
    if flags & WGRAD_DEFER_SUM:
        # a deferred split-K sum reads this call's partial outputs at the flush: a workspace of
        # its own, kept until splitk_flush (allocated on the current stream, where the flush runs)
        nb = ws[CONV_BWD_WEIGHT]
        w = torch.empty(nb, dtype=torch.uint8, device=dw[0].device) if nb else None
        if w is not None:
            _DEFERRED_WS.setdefault(torch.cuda.current_stream(dw[0].device).cuda_stream, []).append(w)
        wp, wsz = (ctypes.c_void_p(w.data_ptr()) if w is not None else None), ctypes.c_size_t(nb)
    else:
        wp, wsz = _ws_args(ws[CONV_BWD_WEIGHT], dw[0].device)
    nx, ny = _prod(in_shape), in_shape[0] * oh * ow * w_shape[0]
    check(_lib.lib().adaptseg_conv2d_bwd_weight_x(
        ctypes.byref(d), _pf(dy, ny, "conv2d_bwd_weight dy"), _pc(dyb, ny, "conv2d_bwd_weight dyb"),
        _pf(x, nx, "conv2d_bwd_weight x"), _pc(xb, nx, "conv2d_bwd_weight xb"), _ptrs(dw),
        _ptrs(db) if len(db) else None, flags, wp, wsz, _stream()), "conv2d_bwd_weight")


WGRAD_DEFER_SUM = 64   # adaptseg.h ADAPTSEG_WGRAD_DEFER_SUM
_DEFERRED_WS: dict = {}   # stream handle -> workspaces of the weight gradients whose sums are pending


def splitk_flush(device=None) -> None:
    """adaptseg_splitk_flush on the current stream: launch the split-K sums the weight gradients
    issued with WGRAD_DEFER_SUM left pending on it, then release their workspaces (freed in
    stream order: the caching allocator reuses them only after the sums on this stream)."""
    s = torch.cuda.current_stream(device)
    check(_lib.lib().adaptseg_splitk_flush(ctypes.c_void_p(s.cuda_stream)), "splitk_flush")
    _DEFERRED_WS.pop(s.cuda_stream, None)


def splitk_pending(device=None) -> int:
    n = ctypes.c_int(0)
    s = torch.cuda.current_stream(device)
    check(_lib.lib().adaptseg_splitk_pending(ctypes.c_void_p(s.cuda_stream), ctypes.byref(n)), "splitk_pending")
    return n.value


# ---- batch norm (x as [rows, C]: the NHWC buffer) ------------------------------------------
_BN_WS: dict = {}


def bn_ws_bytes(rows, c):
    v = _BN_WS.get((rows, c))
    if v is None:
        b = ctypes.c_size_t(0)
        check(_lib.lib().adaptseg_bn_workspace_size(rows, c, ctypes.byref(b)), "bn_workspace_size")
        v = _BN_WS[(rows, c)] = b.value
    return v


def _rc(t):
    c = t.shape[-1]
    return t.numel() // c, c


def _fb(t):
    """(fp32 pointer, bf16 pointer) of an activation operand stored as either."""
    if t is None:
        return None, None
    return (None, _p(t)) if t.dtype == torch.bfloat16 else (_p(t), None)


@_op("bn_fwd_train(Tensor x, Tensor? weight, Tensor? bias, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
     "Tensor? res, Tensor(c!)? y, Tensor(f!)? yb, Tensor(g!)? ybits, Tensor(d!) mean, Tensor(e!) invstd, "
     "float momentum, float eps, int act) -> ()")
def _bn_fwd_train(x, weight, bias, running_mean, running_var, res, y, yb, ybits, mean, invstd, momentum, eps, act):
    """x / res: fp32 or bf16 (bf16 activation storage, config c5); ybits: the ReLU mask bitmap of y
    (int32 [rows, C / 32]) or None."""
    rows, c = _rc(x)
    n = rows * c
    wp, wsz = _ws_args(bn_ws_bytes(rows, c), x.device)
    check(_lib.lib().adaptseg_bn_fwd_train_xm(
        rows, c, *_pfb(x, n, "bn_fwd_train x"), _p(weight), _p(bias), _p(running_mean), _p(running_var),
        float(momentum), float(eps), _p(mean), _p(invstd), *_pfb(res, n, "bn_fwd_train res"),
        _pf(y, n, "bn_fwd_train y"), _pc(yb, n, "bn_fwd_train yb"), _pbits(ybits, n, "bn_fwd_train ybits"),
        int(act), wp, wsz, _stream()), "bn_fwd_train")


@_op("bn_fwd_train_tiles(Tensor x, Tensor stats, int ntiles, Tensor? weight, Tensor? bias, "
     "Tensor(a!)? running_mean, Tensor(b!)? running_var, Tensor? res, Tensor(c!)? y, Tensor(f!)? yb, "
     "Tensor(g!)? ybits, Tensor(d!) mean, Tensor(e!) invstd, float momentum, float eps, int act) -> ()")
def _bn_fwd_train_tiles(x, stats, ntiles, weight, bias, running_mean, running_var, res, y, yb, ybits, mean, invstd,
                        momentum, eps, act):
    rows, c = _rc(x)
    n = rows * c
    check(_lib.lib().adaptseg_bn_fwd_train_tiles_xm(
        rows, c, _p(stats), int(ntiles), *_pfb(x, n, "bn_fwd_train_tiles x"), _p(weight), _p(bias),
        _p(running_mean), _p(running_var), float(momentum), float(eps), _p(mean), _p(invstd),
        *_pfb(res, n, "bn_fwd_train_tiles res"), _pf(y, n, "bn_fwd_train_tiles y"),
        _pc(yb, n, "bn_fwd_train_tiles yb"), _pbits(ybits, n, "bn_fwd_train_tiles ybits"), int(act), _stream()),
        "bn_fwd_train_tiles")


@_op("bn_fwd_infer(Tensor x, Tensor? weight, Tensor? bias, Tensor running_mean, Tensor running_var, "
     "Tensor? res, Tensor(a!)? y, Tensor(b!)? yb, Tensor(c!)? ybits, float eps, int act) -> ()")
def _bn_fwd_infer(x, weight, bias, running_mean, running_var, res, y, yb, ybits, eps, act):
    rows, c = _rc(x)
    n = rows * c
    check(_lib.lib().adaptseg_bn_fwd_infer_xm(
        rows, c, *_pfb(x, n, "bn_fwd_infer x"), _p(weight), _p(bias), _p(running_mean), _p(running_var),
        float(eps), *_pfb(res, n, "bn_fwd_infer res"), _pf(y, n, "bn_fwd_infer y"), _pc(yb, n, "bn_fwd_infer yb"),
        _pbits(ybits, n, "bn_fwd_infer ybits"), int(act), _stream()), "bn_fwd_infer")


@_op("bn_bwd(Tensor dy, Tensor? dybits, Tensor? y, Tensor? x, Tensor? weight, Tensor? bias, Tensor? mean, "
     "Tensor invstd, Tensor(a!)? dx, Tensor(c!)? dxb, Tensor(b!)? dres, int act, bool train) -> ()")
def _bn_bwd(dy, dybits, y, x, weight, bias, mean, invstd, dx, dxb, dres, act, train):
    """y / x (the saved activations): fp32 or bf16; dy and dres fp32, or both bf16 (bf16 gradient
    storage, adaptseg_bn_bwd_xg); dx fp32; dybits: a mask bitmap applied to dy (or None)."""
    rows, c = _rc(dy)
    n = rows * c
    wp, wsz = _ws_args(bn_ws_bytes(rows, c) if train else 0, dy.device)
    check(_lib.lib().adaptseg_bn_bwd_xg(
        rows, c, *_pfb(dy, n, "bn_bwd dy"), _pbits(dybits, n, "bn_bwd dybits"), *_pfb(y, n, "bn_bwd y"),
        *_pfb(x, n, "bn_bwd x"), _p(weight), _p(bias), _p(mean), _p(invstd), _pf(dx, n, "bn_bwd dx"),
        _pc(dxb, n, "bn_bwd dxb"), *_pfb(dres, n, "bn_bwd dres"), int(act), 1 if train else 0, wp, wsz, _stream()),
        "bn_bwd")


@_op("bn_bwd_sums(Tensor dy, Tensor? dybits, Tensor? y, Tensor? x, Tensor? weight, Tensor? bias, Tensor mean, "
     "Tensor invstd, Tensor(a!)? dx, Tensor(c!)? dxb, Tensor(b!)? dres, int act, Tensor partial, int ntiles) -> ()")
def _bn_bwd_sums(dy, dybits, y, x, weight, bias, mean, invstd, dx, dxb, dres, act, partial, ntiles):
    """bn_bwd in train mode whose reduction the producing data gradient's epilogue already did
    (conv2d_bwd_data_bnsum): adaptseg_bn_bwd_sums."""
    rows, c = _rc(dy)
    n = rows * c
    if partial.dtype != torch.float32 or partial.numel() != 2 * c * ntiles:
        raise RuntimeError(f"bn_bwd_sums: partial must be float32 [2][{c}][{ntiles}]")
    wp, wsz = _ws_args(bn_ws_bytes(rows, c), dy.device)
    check(_lib.lib().adaptseg_bn_bwd_sums(
        rows, c, *_pfb(dy, n, "bn_bwd_sums dy"), _pbits(dybits, n, "bn_bwd_sums dybits"), *_pfb(y, n, "bn_bwd_sums y"),
        *_pfb(x, n, "bn_bwd_sums x"), _p(weight), _p(bias), _p(mean), _p(invstd), _pf(dx, n, "bn_bwd_sums dx"),
        _pc(dxb, n, "bn_bwd_sums dxb"), *_pfb(dres, n, "bn_bwd_sums dres"), int(act), _p(partial), int(ntiles), wp,
        wsz, _stream()), "bn_bwd_sums")


@_op("bn_bwd_affine(Tensor dy, Tensor? y, Tensor x, Tensor? weight, Tensor? bias, Tensor mean, "
     "Tensor invstd, Tensor(a!) dx, int act, Tensor(b!)? dweight, Tensor(c!)? dbias) -> ()")
def _bn_bwd_affine(dy, y, x, weight, bias, mean, invstd, dx, act, dweight, dbias):
    rows, c = _rc(dy)
    wp, wsz = _ws_args(bn_ws_bytes(rows, c), dy.device)
    check(_lib.lib().adaptseg_bn_bwd_affine(
        rows, c, _p(dy), _p(y), _p(x), _p(weight), _p(bias), _p(mean), _p(invstd), _p(dx), None, int(act),
        _p(dweight), _p(dbias), wp, wsz, _stream()), "bn_bwd_affine")


# ---- warper -------------------------------------------------------------------------------
@_op("up2_relu_cat_fwd(Tensor? s, Tensor d, Tensor(a!) out) -> ()")
def _up2_relu_cat_fwd(s, d, out):
    n, h, w, cd = d.shape
    cs = 0 if s is None else s.shape[-1]
    check(_lib.lib().adaptseg_up2_relu_cat_fwd(n, h, w, cs, cd, _p(s), _p(d), _p(out), _stream()),
          "up2_relu_cat_fwd")


@_op("up2_relu_cat_bwd(Tensor? s, Tensor d, Tensor dout, Tensor(a!)? ds, Tensor(b!) dd) -> ()")
def _up2_relu_cat_bwd(s, d, dout, ds, dd):
    n, h, w, cd = d.shape
    cs = 0 if s is None else s.shape[-1]
    check(_lib.lib().adaptseg_up2_relu_cat_bwd(n, h, w, cs, cd, _p(s), _p(d), _p(dout), _p(ds), _p(dd),
                                               _stream()), "up2_relu_cat_bwd")


@_op("grid_warp_fwd(Tensor flow, Tensor? x1, Tensor x2, Tensor(a!)? y1, Tensor(b!) y2) -> ()")
def _grid_warp_fwd(flow, x1, x2, y1, y2):
    n, h, w, c = x2.shape
    check(_lib.lib().adaptseg_grid_warp_fwd(n, c, h, w, flow.shape[-1], _p(flow), _p(x1), _p(x2), _p(y1),
                                            _p(y2), _stream()), "grid_warp_fwd")


@_op("grid_warp_bwd(Tensor flow, Tensor? x1, Tensor? x2, Tensor? dy1, Tensor? dy2, Tensor(a!)? dflow, "
     "Tensor(b!)? dx1, Tensor(c!)? dx2) -> ()")
def _grid_warp_bwd(flow, x1, x2, dy1, dy2, dflow, dx1, dx2):
    ref = dy2 if dy2 is not None else dy1
    n, h, w, c = ref.shape
    nbytes = 0
    if dx1 is not None or dx2 is not None:
        b = ctypes.c_size_t(0)
        check(_lib.lib().adaptseg_grid_warp_bwd_workspace_size(n, c, h, w, ctypes.byref(b)),
              "grid_warp_bwd_workspace_size")
        nbytes = b.value
    wp, wsz = _ws_args(nbytes, ref.device)
    check(_lib.lib().adaptseg_grid_warp_bwd(
        n, c, h, w, flow.shape[-1], _p(flow), _p(x1), _p(x2), _p(dy1), _p(dy2), _p(dflow), _p(dx1), _p(dx2),
        wp, wsz, _stream()), "grid_warp_bwd")


# ---- pooling / interpolation / softmax / losses ------------------------------------------
@_op("maxpool2d_fwd(Tensor x, Tensor(a!) y, Tensor(b!) argmax, Tensor(c!)? y_terms, int k, int s, int p) -> ()")
def _maxpool2d_fwd(x, y, argmax, y_terms, k, s, p):
    """y_terms: the pooled output's F32X3 term images [n, oh, ow, 3, c] (bf16) or None."""
    n, h, w, c = x.shape
    oh, ow = y.shape[1], y.shape[2]
    check(_lib.lib().adaptseg_maxpool2d_fwd_x(n, c, h, w, oh, ow, k, s, p, _p(x), _p(y), _p(argmax), _p(y_terms),
                                              _stream()), "maxpool2d_fwd")


@_op("maxpool2d_bwd(Tensor dy, Tensor argmax, Tensor(a!) dx, Tensor(b!)? dx_terms, int k, int s, int p) -> ()")
def _maxpool2d_bwd(dy, argmax, dx, dx_terms, k, s, p):
    """dx_terms: the routed gradient's F32X3 term images [n, h, w, 3, c] (bf16) or None."""
    n, oh, ow, c = dy.shape
    h, w = dx.shape[1], dx.shape[2]
    check(_lib.lib().adaptseg_maxpool2d_bwd_x(n, c, h, w, oh, ow, k, s, p, _p(dy), _p(argmax), _p(dx), _p(dx_terms),
                                              _stream()), "maxpool2d_bwd")


@_op("upsample_bilinear_fwd(Tensor x, Tensor(a!) y) -> ()")
def _upsample_bilinear_fwd(x, y):
    n, h, w, c = x.shape
    check(_lib.lib().adaptseg_upsample_bilinear_fwd(n, c, h, w, y.shape[1], y.shape[2], _p(x), _p(y), _stream()),
          "upsample_bilinear_fwd")


@_op("upsample_bilinear_bwd(Tensor dy, Tensor(a!) dx, bool accumulate) -> ()")
def _upsample_bilinear_bwd(dy, dx, accumulate):
    n, oh, ow, c = dy.shape
    h, w = dx.shape[1], dx.shape[2]
    wp, wsz = _ws_args(n * oh * w * c * 4, dy.device)
    check(_lib.lib().adaptseg_upsample_bilinear_bwd(n, c, h, w, oh, ow, _p(dy), _p(dx),
                                                    _lib.EPI_ACCUMULATE if accumulate else 0, wp, wsz,
                                                    _stream()), "upsample_bilinear_bwd")


@_op("softmax_fwd(Tensor x, Tensor(a!) y) -> ()")
def _softmax_fwd(x, y):
    rows, c = _rc(x)
    check(_lib.lib().adaptseg_softmax_fwd(rows, c, _p(x), _p(y), _stream()), "softmax_fwd")


@_op("softmax_bwd(Tensor y, Tensor dy, Tensor(a!) dx, bool accumulate) -> ()")
def _softmax_bwd(y, dy, dx, accumulate):
    rows, c = _rc(y)
    check(_lib.lib().adaptseg_softmax_bwd(rows, c, _p(y), _p(dy), _p(dx),
                                          _lib.EPI_ACCUMULATE if accumulate else 0, _stream()), "softmax_bwd")


@_op("softmax_ce_fwd(Tensor logits, Tensor labels, int ignore, Tensor? weight, Tensor(a!) out) -> ()")
def _softmax_ce_fwd(logits, labels, ignore, weight, out):
    rows, c = _rc(logits)
    b = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_ce_workspace_size(rows, ctypes.byref(b)), "ce_workspace_size")
    wp, wsz = _ws_args(b.value, logits.device)
    check(_lib.lib().adaptseg_softmax_ce_fwd(rows, c, _p(logits), _p(labels), int(ignore), _p(weight), _p(out),
                                             wp, wsz, _stream()), "softmax_ce_fwd")


@_op("softmax_ce_bwd(Tensor logits, Tensor labels, Tensor out, Tensor grad_loss, int ignore, Tensor? weight, "
     "Tensor(a!) dlogits, bool accumulate) -> ()")
def _softmax_ce_bwd(logits, labels, out, grad_loss, ignore, weight, dlogits, accumulate):
    rows, c = _rc(logits)
    check(_lib.lib().adaptseg_softmax_ce_bwd(rows, c, _p(logits), _p(labels), int(ignore), _p(weight), _p(out),
                                             _p(grad_loss), _p(dlogits),
                                             _lib.EPI_ACCUMULATE if accumulate else 0, _stream()),
          "softmax_ce_bwd")


@_op("adv_loss_fwd(Tensor x, float target, int kind, Tensor(a!) loss) -> ()")
def _adv_loss_fwd(x, target, kind, loss):
    n = x.numel()
    b = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_adv_workspace_size(n, ctypes.byref(b)), "adv_workspace_size")
    wp, wsz = _ws_args(b.value, x.device)
    check(_lib.lib().adaptseg_adv_loss_fwd(n, _p(x), float(target), int(kind), _p(loss), wp, wsz, _stream()),
          "adv_loss_fwd")


@_op("adv_loss_bwd(Tensor x, float target, int kind, Tensor grad_loss, Tensor(a!) dx, bool accumulate) -> ()")
def _adv_loss_bwd(x, target, kind, grad_loss, dx, accumulate):
    check(_lib.lib().adaptseg_adv_loss_bwd(x.numel(), _p(x), float(target), int(kind), _p(grad_loss), _p(dx),
                                           _lib.EPI_ACCUMULATE if accumulate else 0, _stream()), "adv_loss_bwd")


# ---- optimisers and plumbing ----------------------------------------------------------------
@_op("sgd_step(Tensor(a!) param, Tensor grad, Tensor(b!) momentum_buffer, float lr, float momentum, "
     "float weight_decay, float grad_scale, int multiplicity, bool first_step) -> ()")
def _sgd_step(param, grad, momentum_buffer, lr, momentum, weight_decay, grad_scale, multiplicity, first_step):
    check(_lib.lib().adaptseg_sgd_step(param.numel(), _p(param), _p(grad), _p(momentum_buffer), float(lr),
                                       float(momentum), float(weight_decay), float(grad_scale), int(multiplicity),
                                       1 if first_step else 0, _stream()), "sgd_step")


@_op("adam_step(Tensor(a!) param, Tensor grad, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, float lr, "
     "float beta1, float beta2, float eps, int step, float grad_scale) -> ()")
def _adam_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, step, grad_scale):
    check(_lib.lib().adaptseg_adam_step(param.numel(), _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq),
                                        float(lr), float(beta1), float(beta2), float(eps), int(step),
                                        float(grad_scale), _stream()), "adam_step")


@_op("zero(Tensor(a!) t) -> ()")
def _zero(t):
    check(_lib.lib().adaptseg_zero(_p(t), t.numel() * t.element_size(), _stream()), "zero")


@_op("to_nhwc(Tensor x, Tensor(a!) out) -> ()")
def _to_nhwc(x, out):
    n, c, h, w = x.shape
    st = (ctypes.c_int64 * 4)(*x.stride())
    check(_lib.lib().adaptseg_to_nhwc(n, c, h, w, st, _p(x), _p(out), _stream()), "to_nhwc")


@_op("to_nhwc_pad(Tensor x, Tensor(a!) out, bool accumulate) -> ()")
def _to_nhwc_pad(x, out, accumulate):
    """out [n, h, w, c_dst] (=|+=) x (NCHW-shaped, any strides), channels >= c zero."""
    n, c, h, w = x.shape
    st = (ctypes.c_int64 * 4)(*x.stride())
    check(_lib.lib().adaptseg_to_nhwc_pad(n, c, h, w, st, _p(x), out.shape[-1], _p(out),
                                          _lib.EPI_ACCUMULATE if accumulate else 0, _stream()), "to_nhwc_pad")


@_op("axpy(float alpha, Tensor src, Tensor(a!) dst, bool accumulate) -> ()")
def _axpy(alpha, src, dst, accumulate):
    check(_lib.lib().adaptseg_axpy(src.numel(), float(alpha), _p(src), _p(dst),
                                   _lib.EPI_ACCUMULATE if accumulate else 0, _stream()), "axpy")


@_op("add_i64(Tensor(a!) t, int v) -> ()")
def _add_i64(t, v):
    check(_lib.lib().adaptseg_add_i64(_p(t), t.numel(), int(v), _stream()), "add_i64")


# ---- input pipeline and evaluation -----------------------------------------------
@_op("gta5_preprocess(Tensor images, float[] mean, Tensor(a!) out, Tensor? labels, Tensor? lut, "
     "Tensor(b!)? labels_out) -> ()")
def _gta5_preprocess(images, mean, out, labels, lut, labels_out):
    n, h, w, _ = images.shape
    oh, ow = out.shape[2], out.shape[3]
    b = ctypes.c_size_t(0)
    check(_lib.lib().adaptseg_preprocess_workspace_size(n, h, w, oh, ow, ctypes.byref(b)),
          "preprocess_workspace_size")
    wp, wsz = _ws_args(b.value, images.device)
    check(_lib.lib().adaptseg_gta5_preprocess(
        n, h, w, oh, ow, _p(images), float(mean[0]), float(mean[1]), float(mean[2]), _p(out), _p(labels),
        _p(lut) if labels is not None else None, _p(labels_out), wp, wsz, _stream()), "gta5_preprocess")


@_op("upsample_argmax(Tensor x, Tensor(a!) out) -> ()")
def _upsample_argmax(x, out):
    n, h, w, c = x.shape
    check(_lib.lib().adaptseg_upsample_argmax(n, c, h, w, out.shape[1], out.shape[2], _p(x), _p(out), _stream()),
          "upsample_argmax")


@_op("confusion_hist(Tensor gt_ids, Tensor lut, Tensor pred, int num_classes, Tensor(a!) hist) -> ()")
def _confusion_hist(gt_ids, lut, pred, num_classes, hist):
    check(_lib.lib().adaptseg_confusion_hist(gt_ids.numel(), _p(gt_ids), _p(lut), _p(pred), int(num_classes),
                                             _p(hist), _stream()), "confusion_hist")


class _Overloads:
    """torch.ops.adaptseg.<name>.default for every op (skips the packet's overload lookup)."""


OPS = _Overloads()
for _n in NAMES:
    setattr(OPS, _n, getattr(torch.ops.adaptseg, _n).default)
