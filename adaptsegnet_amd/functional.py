"""Autograd Functions for the step's memory-bound ops (softmax, CE, adversarial losses).

Tensors at this boundary are NCHW-shaped, as in the reference; internally they are NHWC
(channels_last) buffers, and a non-channels_last input is converted by the native
``adaptseg_to_nhwc`` kernel.  Reference call sites:
  F.softmax(pred)                               train_gta2cityscapes_multi.py:423,442,454,617-618
  nn.CrossEntropyLoss(ignore_index=255)         train_gta2cityscapes_multi.py:359,546,599-600
  CrossEntropy2d                                utils/loss.py:14-36
  BCEWithLogitsLoss / MSELoss vs const target   train_gta2cityscapes_multi.py:542-545,620-624
  nn.Upsample(bilinear, align_corners=True)     train_gta2cityscapes_multi.py:237-238 (interp),
                                                model/deeplab_multi.py:188-189
"""
from __future__ import annotations

import torch

from . import kernels as K

BCE, MSE = 0, 1


def _check(x, what):
    if not x.is_cuda:
        raise RuntimeError(f"{what}: adaptsegnet_amd ops run on the HIP device only (got {x.device})")
    if x.dtype != torch.float32:
        raise RuntimeError(f"{what}: expected float32, got {x.dtype}")


class _Softmax2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = K.softmax_fwd(K.nhwc_view(x))
        ctx.save_for_backward(y)
        return K.as_nchw(y)

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        return K.as_nchw(K.softmax_bwd(y, K.nhwc_view(g)))


def softmax2d(x: torch.Tensor) -> torch.Tensor:
    """Softmax over the channel dim of an [N, C, H, W] tensor (F.softmax's implicit dim=1)."""
    _check(x, "softmax2d")
    return _Softmax2d.apply(x)


class _CrossEntropy2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore, weight, total):
        x = K.nhwc_view(logits)
        out = K.ce_fwd(x, labels, ignore, weight)   # [mean, denominator]
        ctx.save_for_backward(x, labels, out, weight)
        ctx.ignore, ctx.total = ignore, total
        if total:   # reduction='sum': mean * denominator; an empty selection sums to 0
            return torch.where(out[1] > 0, out[0] * out[1], torch.zeros_like(out[0]))
        return out[0]

    @staticmethod
    def backward(ctx, g):
        x, labels, out, weight = ctx.saved_tensors
        if g.dim() == 0:
            g = g.reshape(1)
        if ctx.total:   # d(sum)/dlogits = denominator * d(mean)/dlogits
            g = g * out[1:2]
        dl = K.ce_bwd(x, labels, out, g.contiguous(), ctx.ignore, weight)
        return K.as_nchw(dl), None, None, None, None


def cross_entropy2d(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = 255,
                    weight: torch.Tensor | None = None, reduction: str = "mean") -> torch.Tensor:
    """Softmax cross entropy over pixels whose label is >= 0 and != ignore_index.

    logits: [N, C, H, W] fp32; labels: [N, H, W] int64.  reduction 'mean' (weighted by
    ``weight[label]`` when given) or 'sum'.  Returns a 0-dim device tensor; an all-ignored
    batch gives NaN for the mean (like the reference) and 0 for the sum (F.cross_entropy).
    """
    if reduction not in ("mean", "sum"):
        raise ValueError(f"cross_entropy2d: reduction {reduction!r} (expected 'mean' or 'sum')")
    _check(logits, "cross_entropy2d")
    if labels.dtype != torch.int64:
        raise RuntimeError(f"cross_entropy2d: labels must be int64 (got {labels.dtype})")
    n, c, h, w = logits.shape
    if labels.shape != (n, h, w):
        raise RuntimeError(f"cross_entropy2d: labels {tuple(labels.shape)} vs logits {tuple(logits.shape)}")
    labels = labels.contiguous()
    if weight is not None:
        weight = weight.to(device=logits.device, dtype=torch.float32).contiguous()
    return _CrossEntropy2d.apply(logits, labels, int(ignore_index), weight, reduction == "sum")


class _AdvLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target, kind):
        xc = x.contiguous() if not (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)) else x
        loss = K.adv_fwd(xc, target, kind)
        ctx.save_for_backward(xc)
        ctx.target, ctx.kind = target, kind
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        if g.dim() == 0:
            g = g.reshape(1)
        return K.adv_bwd(x, ctx.target, ctx.kind, g.contiguous()), None, None


def adv_loss(d_out: torch.Tensor, target: float, kind: int) -> torch.Tensor:
    """mean(BCEWithLogits(d_out, target)) (kind=BCE) or mean((d_out-target)^2) (kind=MSE)."""
    _check(d_out, "adv_loss")
    return _AdvLoss.apply(d_out, float(target), int(kind))


def bce_with_logits_const(d_out, target: float):
    return adv_loss(d_out, target, BCE)


def mse_const(d_out, target: float):
    return adv_loss(d_out, target, MSE)


class _Interp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        xv = K.nhwc_view(x)
        ctx.hw = (xv.shape[1], xv.shape[2])
        return K.as_nchw(K.upsample_fwd(xv, oh, ow))

    @staticmethod
    def backward(ctx, g):
        h, w = ctx.hw
        return K.as_nchw(K.upsample_bwd(K.nhwc_view(g), h, w)), None, None


def interp(x: torch.Tensor, size) -> torch.Tensor:
    """``nn.Upsample(size=(H, W), mode='bilinear', align_corners=True)(x)`` for [N, C, h, w]."""
    _check(x, "interp")
    return _Interp.apply(x, int(size[0]), int(size[1]))
