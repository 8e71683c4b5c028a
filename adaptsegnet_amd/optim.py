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
                self._started.update(o for o in A.offsets if a <= o < b)

    # -- resume (checkpoint.py) --------------------------------------------------------------
    def state_dict(self, names):
        """{param name: momentum buffer (reference layout)} for parameters that have one,
        plus the LRs.  ``names``: arena index -> state_dict key of the model."""
        A = self.model.arena
        st = {}
        if A is not None and self._buf is not None:
            for i, (p, off) in enumerate(zip(A.params, A.offsets)):
                if off in self._started:
                    st[names[i]] = A._view(self._buf, p, off).detach().cpu().contiguous()
        return {"momentum_buffer": st, "lr": [g["lr"] for g in self.param_groups]}

    @torch.no_grad()
    def load_state_dict(self, state, names):
        A = self.model.arena
        self._buf = torch.zeros(A.numel, dtype=torch.float32, device=A.device)
        self._arena_id = id(A)
        self._started = set()
        bufs = state["momentum_buffer"]
        for i, (p, off) in enumerate(zip(A.params, A.offsets)):
            if names[i] in bufs:
                A._view(self._buf, p, off).copy_(bufs[names[i]])
                self._started.add(off)
        for g, lr in zip(self.param_groups, state["lr"]):
            g["lr"] = lr


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
                for o in A.offsets:
                    if a <= o < b:
                        self._steps[o] = st
                K.adam_step(A.data[a:b], A.grad[a:b], self._m[a:b], self._v[a:b], lr,
                            self.betas[0], self.betas[1], self.eps, st, grad_scale)

    # -- resume (checkpoint.py) --------------------------------------------------------------
    def state_dict(self, names):
        """torch.optim.Adam-like per-parameter state keyed by the model's state_dict names."""
        A = self.model.arena
        st = {}
        if A is not None and self._m is not None:
            for i, (p, off) in enumerate(zip(A.params, A.offsets)):
                if off in self._steps:
                    st[names[i]] = {"step": self._steps[off],
                                    "exp_avg": A._view(self._m, p, off).detach().cpu().contiguous(),
                                    "exp_avg_sq": A._view(self._v, p, off).detach().cpu().contiguous()}
        return {"state": st, "lr": [g["lr"] for g in self.param_groups]}

    @torch.no_grad()
    def load_state_dict(self, state, names):
        A = self.model.arena
        self._m = torch.zeros(A.numel, dtype=torch.float32, device=A.device)
        self._v = torch.zeros(A.numel, dtype=torch.float32, device=A.device)
        self._arena_id = id(A)
        self._steps = {}
        for i, (p, off) in enumerate(zip(A.params, A.offsets)):
            s = state["state"].get(names[i])
            if s is not None:
                A._view(self._m, p, off).copy_(s["exp_avg"])
                A._view(self._v, p, off).copy_(s["exp_avg_sq"])
                self._steps[off] = int(s["step"])
        for g, lr in zip(self.param_groups, state["lr"]):
            g["lr"] = lr
