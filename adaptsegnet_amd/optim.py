"""Fused optimisers over a model's parameter arena (one HIP launch per contiguous range).

``SGD(model, lr, momentum, weight_decay)`` replaces
``optim.SGD(model.optim_parameters(args), lr=..., momentum=..., weight_decay=...)``
(train_gta2cityscapes_multi.py:532-533), including the reference's duplicate-parameter
multiplicity and its skipping of parameters whose ``.grad`` is None (layer5 in the
single-level step).  ``Adam(model_D, lr, betas)`` replaces ``optim.Adam(model_D.parameters(),
lr=..., betas=(0.9, 0.99))`` (:536-540).  Both expose ``param_groups[i]['lr']`` so the
reference's ``adjust_learning_rate`` / ``adjust_learning_rate_D`` (:166-177) work unchanged.

``step(grad_scale=s)`` multiplies every gradient by ``s`` first — the 1/world_size of a
data-parallel SUM all-reduce is folded in here instead of a separate scaling pass.
"""
from __future__ import annotations

import torch

from . import kernels as K


def lr_poly(base_lr, it, max_iter, power):
    """train_gta2cityscapes_multi.py:162-163."""
    return base_lr * ((1 - float(it) / max_iter) ** power)


class SGD:
    def __init__(self, model, lr, momentum=0.9, weight_decay=5e-4, lr_mult_10x=True):
        self.model = model
        self.momentum, self.weight_decay = float(momentum), float(weight_decay)
        self.param_groups = [{"lr": float(lr)}, {"lr": float(lr) * (10.0 if lr_mult_10x else 1.0)}]
        self._buf = None
        self._arena_id = None
        self._started = set()  # arena offsets whose momentum buffer exists (torch state)

    def zero_grad(self, set_to_none: bool = True):
        if self.model.arena is not None:
            self.model.arena.zero_grad(set_to_none)

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        A = self.model.arena
        if A is None:
            return
        if self._buf is None or self._arena_id != id(A):
            self._buf = torch.zeros(A.numel, dtype=torch.float32, device=A.device)
            self._arena_id = id(A)
            self._started = set()
        for seg in A.segments:
            lr = self.param_groups[seg.group]["lr"]
            for a, b in A.runs(seg):
                first = a not in self._started
                K.sgd_step(A.data[a:b], A.grad[a:b], self._buf[a:b], lr, self.momentum,
                           self.weight_decay, grad_scale, seg.mult, first)
                self._started.add(a)


class Adam:
    def __init__(self, model, lr, betas=(0.9, 0.99), eps=1e-8):
        self.model = model
        self.betas, self.eps = (float(betas[0]), float(betas[1])), float(eps)
        self.param_groups = [{"lr": float(lr)}]
        self._m = self._v = None
        self._arena_id = None
        self._steps = {}

    def zero_grad(self, set_to_none: bool = True):
        if self.model.arena is not None:
            self.model.arena.zero_grad(set_to_none)

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        A = self.model.arena
        if A is None:
            return
        if self._m is None or self._arena_id != id(A):
            self._m = torch.zeros(A.numel, dtype=torch.float32, device=A.device)
            self._v = torch.zeros(A.numel, dtype=torch.float32, device=A.device)
            self._arena_id = id(A)
            self._steps = {}
        lr = self.param_groups[0]["lr"]
        for seg in A.segments:
            for a, b in A.runs(seg):
                st = self._steps.get(a, 0) + 1
                self._steps[a] = st
                K.adam_step(A.data[a:b], A.grad[a:b], self._m[a:b], self._v[a:b], lr,
                            self.betas[0], self.betas[1], self.eps, st, grad_scale)
