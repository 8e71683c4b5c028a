"""DeeplabVGG (VGG16 with dilated conv5, fc6/fc7 as atrous convs, ASPP head) on the HIP engine.

Drop-in for /root/reference/model/deeplab_vgg.py:24-54 (benchmark config c4, the
non-residual conv path):

* ``features`` is the VGG16 (cfg "D") feature stack with pool4 and pool5 removed
  (:32-33, old indices 23 and 30), so the three conv5 layers land on indices 23/25/27 and
  get dilation 2 / padding 2 (:35-37); then fc6 = 3x3 d4 512->1024 (index 29) and
  fc7 = 3x3 d4 1024->1024 (index 31), each followed by ReLU (:39-42).  Every conv carries a
  bias; ReLU is fused into the conv epilogue, MaxPool2d(2, 2) runs as its own kernel.
* ``classifier`` is the 4-branch ``Classifier_Module`` (:7-21) — but its forward returns
  inside the loop (:19-21), so only branches 0 and 1 (d6 + d12) are summed.  The engine
  runs exactly that as one 2-segment conv; branches 2 and 3 keep their parameters (and
  state_dict keys) and never receive a gradient, as upstream.
* ``forward(x)`` returns the [N, C, H/8, W/8] map; the caller upsamples (the reference's
  ``interp``), e.g. with ``adaptsegnet_amd.functional.interp``.
* ``optim_parameters(args)`` returns ``self.parameters()`` (one LR group, :53-54).

Init follows what the reference gets from ``torchvision.models.vgg16()`` (kaiming-normal
fan_out conv weights, zero biases), ``nn.Conv2d`` defaults for fc6/fc7 and N(0, 0.01) for the
classifier weights (:13-14).  ``pretrained=True`` loads a torchvision-layout VGG16 state
dict with ``torch.load(..., weights_only=True)`` and applies the reference's index shift.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import engine
from .deeplab_multi import Classifier_Module
from .layers import Conv2d, ParamArena

# VGG16 cfg "D" after removing pool4/pool5: ('C', cin, cout, dilation) / ('P',) / ('R',)
_VGG_FEATURES = (
    ("C", 3, 64, 1), ("R",), ("C", 64, 64, 1), ("R",), ("P",),
    ("C", 64, 128, 1), ("R",), ("C", 128, 128, 1), ("R",), ("P",),
    ("C", 128, 256, 1), ("R",), ("C", 256, 256, 1), ("R",), ("C", 256, 256, 1), ("R",), ("P",),
    ("C", 256, 512, 1), ("R",), ("C", 512, 512, 1), ("R",), ("C", 512, 512, 1), ("R",),
    ("C", 512, 512, 2), ("R",), ("C", 512, 512, 2), ("R",), ("C", 512, 512, 2), ("R",),
)
# torchvision vgg16 feature index -> index in the pool4/pool5-free stack (:32)
_TV_INDEX = {i: i for i in range(23)}
_TV_INDEX.update({i: i - 1 for i in range(24, 30)})


class DeeplabVGG(nn.Module):
    single_output = True  # forward returns one un-upsampled map (the trainer upsamples it)

    def __init__(self, num_classes, vgg16_caffe_path=None, pretrained=False):
        super().__init__()
        mods = []
        for spec in _VGG_FEATURES:
            if spec[0] == "C":
                _, ci, co, d = spec
                conv = Conv2d(ci, co, kernel_size=3, padding=d, dilation=d)
                with torch.no_grad():  # torchvision VGG init: kaiming_normal_(fan_out, relu), bias 0
                    conv.weight.normal_(0.0, math.sqrt(2.0 / (co * 9)))
                    conv.bias.zero_()
                mods.append(conv)
            elif spec[0] == "R":
                mods.append(nn.ReLU(inplace=True))
            else:
                mods.append(nn.MaxPool2d(kernel_size=2, stride=2))
        fc6 = Conv2d(512, 1024, kernel_size=3, padding=4, dilation=4)
        fc7 = Conv2d(1024, 1024, kernel_size=3, padding=4, dilation=4)
        self.features = nn.Sequential(*(mods + [fc6, nn.ReLU(inplace=True), fc7, nn.ReLU(inplace=True)]))
        self.classifier = Classifier_Module(1024, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)
        if pretrained:
            self._load_vgg16(vgg16_caffe_path)
        self._arena = None
        self._arena_valid = False

    def _load_vgg16(self, path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        own = self.state_dict()
        with torch.no_grad():
            for k, v in sd.items():
                parts = k.split(".")
                if parts[0] != "features" or int(parts[1]) not in _TV_INDEX:
                    continue  # pool indices and the VGG fc classifier are not used (:30-33)
                key = f"features.{_TV_INDEX[int(parts[1])]}.{parts[2]}"
                own[key].copy_(v)

    # -- the layer program the engine runs ------------------------------------------------
    def conv_program(self):
        """[(conv, pool_after)] in order: fused conv+bias+ReLU, then an optional 2x2 pool."""
        feats = list(self.features)
        prog = []
        for i, m in enumerate(feats):
            if isinstance(m, Conv2d):
                pool = i + 2 < len(feats) and isinstance(feats[i + 2], nn.MaxPool2d)
                prog.append((m, pool))
        return prog

    def classifier_branches(self):
        """The branches Classifier_Module.forward actually sums (:17-21): 0 and 1."""
        return list(self.classifier.conv2d_list)[:2]

    def optim_parameters(self, args):
        return self.parameters()

    # -- arena --------------------------------------------------------------------------
    def _apply(self, fn, *args, **kwargs):
        self._arena_valid = False
        return super()._apply(fn, *args, **kwargs)

    def _ensure_arena(self, device):
        if self._arena_valid and self._arena is not None and self._arena.device == device:
            return
        self._arena = ParamArena([(list(self.parameters()), 0, 1)], device)
        A = self._arena
        used = [p for conv, _ in self.conv_program() for p in conv.parameters()]
        used += [p for c in self.classifier_branches() for p in c.parameters()]
        self._pidx = {"used": A.index_of([p for p in used if p.requires_grad])}
        self._anchors = {
            True: torch.empty(0, device=device, requires_grad=True),
            False: torch.empty(0, device=device, requires_grad=False),
        }
        self._arena_valid = True

    @property
    def arena(self) -> ParamArena:
        return self._arena

    def forward(self, x):
        return engine.deeplab_vgg_forward(self, x)
