"""Parameter-holding layers with the reference's state_dict names, and the flat arena.

``Conv2d`` / ``BatchNorm2d`` here only HOLD parameters and buffers (same attribute names,
shapes and default init as ``torch.nn.Conv2d`` / ``torch.nn.BatchNorm2d``, so checkpoints
interchange with the reference); their arithmetic is run by the HIP engine
(``adaptsegnet_amd.engine``), never by torch.  Calling them directly raises.

``ParamArena`` packs a module's trainable parameters into one flat fp32 buffer (4-D
weights stored [Cout][KH][KW][Cin], i.e. torch channels_last) with a parallel flat
gradient buffer.  Weight-gradient kernels accumulate straight into it, the gradient
all-reduce is one collective over it, and the optimiser is one fused kernel per LR group.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import kernels as K

_ALIGN = 64  # floats (256 B) between parameters: keeps every float4 load aligned


class Conv2d(nn.Module):
    """Holds nn.Conv2d-compatible ``weight`` [Cout, Cin, KH, KW] (+ ``bias``)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (kernel_size, kernel_size)
        self.stride, self.padding, self.dilation = stride, padding, dilation
        w = torch.empty(out_channels, in_channels, kernel_size, kernel_size)
        self.weight = nn.Parameter(w.contiguous(memory_format=torch.channels_last))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # torch.nn.Conv2d default init: kaiming_uniform_(a=sqrt(5)) == U(-1/sqrt(fan_in), +)
        fan_in = self.in_channels * self.kernel_size[0] * self.kernel_size[1]
        bound = 1.0 / math.sqrt(fan_in)
        with torch.no_grad():
            self.weight.uniform_(-bound, bound)
            if self.bias is not None:
                self.bias.uniform_(-bound, bound)

    def geom(self) -> K.ConvGeom:
        return K.ConvGeom(self.in_channels, self.out_channels, self.kernel_size[0],
                          self.kernel_size[1], self.stride, (self.padding,), (self.dilation,))

    def forward(self, *a, **k):  # pragma: no cover - guard
        raise RuntimeError("adaptsegnet_amd Conv2d is a parameter holder; run the parent module")

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}, dilation={self.dilation}, "
                f"bias={self.bias is not None}")


class BatchNorm2d(nn.Module):
    """Holds nn.BatchNorm2d-compatible weight/bias/running_mean/running_var/num_batches_tracked."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def forward(self, *a, **k):  # pragma: no cover - guard
        raise RuntimeError("adaptsegnet_amd BatchNorm2d is a parameter holder; run the parent module")

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}, affine=True"


class ArenaSegment:
    """A contiguous range of the arena: one LR group and one update multiplicity."""

    __slots__ = ("start", "end", "group", "mult")

    def __init__(self, start, end, group, mult):
        self.start, self.end, self.group, self.mult = start, end, group, mult


class ParamArena:
    """Flat storage for trainable parameters and their gradients.

    ``segments`` is a list of ``(params, group, multiplicity)``: ``group`` indexes the
    optimiser's param_groups (LR), ``multiplicity`` is how many times the reference's
    parameter generator lists each of those parameters (see ``adaptseg_sgd_step``).
    """

    def __init__(self, segments, device):
        self.device = torch.device(device)
        self.params, self.offsets, self.segments = [], [], []
        o = 0
        for params, group, mult in segments:
            start = o
            for p in params:
                self.params.append(p)
                self.offsets.append(o)
                o += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
            if o > start:
                self.segments.append(ArenaSegment(start, o, group, mult))
        self.numel = o
        self.data = torch.zeros(o, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(o, dtype=torch.float32, device=self.device)
        self._grad_views = []
        for p, off in zip(self.params, self.offsets):
            view = self._view(self.data, p, off)
            with torch.no_grad():
                view.copy_(p.data.to(self.device))
            p.data = view
            self._grad_views.append(self._view(self.grad, p, off))

    @staticmethod
    def _view(flat, p, off):
        n = p.numel()
        if p.dim() == 4:
            co, ci, kh, kw = p.shape
            return flat[off:off + n].view(co, kh, kw, ci).permute(0, 3, 1, 2)
        return flat[off:off + n].view(p.shape)

    def valid(self) -> bool:
        base = self.data.data_ptr()
        return all(p.data.data_ptr() == base + 4 * off for p, off in zip(self.params, self.offsets))

    def index_of(self, params) -> list:
        idx = {id(p): i for i, p in enumerate(self.params)}
        return [idx[id(p)] for p in params if id(p) in idx]

    def claim(self, indices) -> None:
        """Give params[indices] arena-backed ``.grad`` before a backward writes them.

        Mirrors torch's AccumulateGrad: a parameter whose ``.grad`` is None starts from
        zero, one whose ``.grad`` already is its arena view keeps accumulating.
        """
        fresh = [i for i in indices
                 if self.params[i].grad is None
                 or self.params[i].grad.data_ptr() != self._grad_views[i].data_ptr()]
        if not fresh:
            return
        if all(p.grad is None for p in self.params):
            K.zero_(self.grad)
        else:
            for i in fresh:
                p, gv = self.params[i], self._grad_views[i]
                if p.grad is None:
                    K.zero_(self.grad[self.offsets[i]:self.offsets[i] + p.numel()])
                else:  # a foreign .grad tensor (user-assigned): adopt its values
                    with torch.no_grad():
                        gv.copy_(p.grad)
        for i in fresh:
            self.params[i].grad = self._grad_views[i]

    def zero_grad(self, set_to_none: bool = True) -> None:
        """optimizer.zero_grad(): grads -> None (torch >= 2 default) or zeros."""
        K.zero_(self.grad)
        for p, gv in zip(self.params, self._grad_views):
            p.grad = None if set_to_none else gv

    def has_grad(self, i) -> bool:
        p = self.params[i]
        return p.grad is not None and p.grad.data_ptr() == self._grad_views[i].data_ptr()

    def runs(self, seg):
        """Contiguous [start, end) ranges of ``seg`` whose params currently hold a gradient."""
        out, cur = [], None
        for i, (p, off) in enumerate(zip(self.params, self.offsets)):
            if off < seg.start or off >= seg.end:
                continue
            if self.has_grad(i):
                end = off + p.numel()
                if cur is not None and cur[1] >= off - _ALIGN and cur[1] <= off:
                    cur[1] = end
                else:
                    cur = [off, end]
                    out.append(cur)
            else:
                cur = None
        return [(a, b) for a, b in out]


def normal_init_(model: nn.Module, std: float = 0.01):
    """ResNetMulti init (model/deeplab_multi.py:144-150): conv weights N(0, std), BN 1/0."""
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, Conv2d):
                m.weight.normal_(0, std)
            elif isinstance(m, BatchNorm2d):
                m.weight.fill_(1)
                m.bias.zero_()
