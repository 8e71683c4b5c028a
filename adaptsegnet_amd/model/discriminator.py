"""FCDiscriminator on the MI355X HIP engine.

Drop-in for /root/reference/model/discriminator.py:5-34: five 4x4 stride-2 pad-1 convs
with bias (num_classes -> ndf -> 2ndf -> 4ndf -> 8ndf -> 1), LeakyReLU(0.2) after the
first four (fused into the conv epilogue), torch.nn.Conv2d default init, identical
state_dict keys (``conv{1..4}.{weight,bias}``, ``classifier.{weight,bias}``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import engine
from .layers import Conv2d, ParamArena


class FCDiscriminator(nn.Module):

    def __init__(self, num_classes, ndf=64):
        super().__init__()
        self.conv1 = Conv2d(num_classes, ndf, kernel_size=4, stride=2, padding=1)
        self.conv2 = Conv2d(ndf, ndf * 2, kernel_size=4, stride=2, padding=1)
        self.conv3 = Conv2d(ndf * 2, ndf * 4, kernel_size=4, stride=2, padding=1)
        self.conv4 = Conv2d(ndf * 4, ndf * 8, kernel_size=4, stride=2, padding=1)
        self.classifier = Conv2d(ndf * 8, 1, kernel_size=4, stride=2, padding=1)
        self.negative_slope = 0.2
        self._arena = None
        self._arena_valid = False

    def _convs(self):
        return (self.conv1, self.conv2, self.conv3, self.conv4, self.classifier)

    def _apply(self, fn, *args, **kwargs):
        self._arena_valid = False
        return super()._apply(fn, *args, **kwargs)

    def _ensure_arena(self, device):
        if self._arena_valid and self._arena is not None and self._arena.device == device:
            return
        self._arena = ParamArena([(list(self.parameters()), 0, 1)], device)
        self._pidx = {"all": list(range(len(self._arena.params)))}
        self._anchors = {
            True: torch.empty(0, device=device, requires_grad=True),
            False: torch.empty(0, device=device, requires_grad=False),
        }
        self._arena_valid = True

    @property
    def arena(self) -> ParamArena:
        return self._arena

    def forward(self, x):
        return engine.discriminator_forward(self, x)
