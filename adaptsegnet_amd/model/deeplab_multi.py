"""DeeplabMulti (ResNet-101 backbone + two ASPP heads) on the MI355X HIP engine.

Drop-in for /root/reference/model/deeplab_multi.py: same class names, constructor and
forward signatures, same module tree and therefore the same ``state_dict()`` keys
(``conv1.weight``, ``bn1.*``, ``layerK.i.conv{1,2,3}.weight``, ``layerK.0.downsample.{0,1}.*``,
``layer{5,6}.conv2d_list.{0..3}.{weight,bias}``), same initialisation and the same
``optim_parameters(args)`` groups.  The arithmetic runs in ``adaptsegnet_amd.engine``.

Reference semantics kept (file:line):
  Bottleneck (1x1 stride on conv1, BN frozen)        model/deeplab_multi.py:59-103
  Classifier_Module (sum of 4 dilated 3x3 + bias)    :106-121
  ResNetMulti layers / init / forward                :124-194
  get_1x_lr_params_NOscale / get_10x_lr_params        :196-231
  optim_parameters (1x and 10x LR groups)            :233-235
  DeeplabMulti(num_classes)                          :258-260
  ResNetMulti.warp (tanh + linspace grid, clamp, grid_sample)  :238-255
Deliberate difference: ``forward`` accepts ``input_size=None`` (then the input's own (W, H) is
used — the reference's multi-level call site train_gta2cityscapes_multi.py:597 omits it and
raises).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import engine
from .layers import BatchNorm2d, Conv2d, ParamArena, normal_init_

affine_par = True


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, dilation=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, kernel_size=1, stride=stride, bias=False)
        self.bn1 = BatchNorm2d(planes)
        padding = dilation
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=1, padding=padding,
                            dilation=dilation, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(planes * 4)
        for bn in (self.bn1, self.bn2, self.bn3):
            for p in bn.parameters():
                p.requires_grad = False
        self.downsample = downsample
        self.stride = stride


class Classifier_Module(nn.Module):
    def __init__(self, inplanes, dilation_series, padding_series, num_classes):
        super().__init__()
        self.conv2d_list = nn.ModuleList()
        for dilation, padding in zip(dilation_series, padding_series):
            self.conv2d_list.append(Conv2d(inplanes, num_classes, kernel_size=3, stride=1,
                                           padding=padding, dilation=dilation, bias=True))
        with torch.no_grad():
            for m in self.conv2d_list:
                m.weight.normal_(0, 0.01)


class ResNetMulti(nn.Module):
    def __init__(self, block, layers, num_classes):
        self.inplanes = 64
        super().__init__()
        self.conv1 = Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNorm2d(64)
        for p in self.bn1.parameters():
            p.requires_grad = False
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=1, dilation=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=1, dilation=4)
        self.layer5 = Classifier_Module(1024, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)
        self.layer6 = Classifier_Module(2048, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)
        normal_init_(self, 0.01)
        self._arena = None
        self._arena_valid = False
        # data parallel: called as hook(unit_ordinal, stream) after the engine launched a
        # backward unit's weight gradients (see _bwd_units), hook(None, stream) at the end
        self._grad_hook = None

    def _make_layer(self, block, planes, blocks, stride=1, dilation=1):
        downsample = None
        if (stride != 1 or self.inplanes != planes * block.expansion or dilation == 2
                or dilation == 4):
            downsample = nn.Sequential(
                Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride,
                       bias=False),
                BatchNorm2d(planes * block.expansion))
            for p in downsample[1].parameters():
                p.requires_grad = False
        layers = [block(self.inplanes, planes, stride, dilation=dilation, downsample=downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, dilation=dilation))
        return nn.Sequential(*layers)

    # -- parameter groups (reference order, reference multiplicity) ------------------
    def get_1x_lr_params_NOscale(self):
        """model/deeplab_multi.py:196-222.  Like the reference this walks ``modules()`` and
        takes the RECURSIVE ``parameters()`` of each, so a block conv weight is yielded 3x
        and a downsample conv weight 4x; torch.optim applies duplicates sequentially."""
        for mod in (self.conv1, self.bn1, self.layer1, self.layer2, self.layer3, self.layer4):
            for m in mod.modules():
                for k in m.parameters():
                    if k.requires_grad:
                        yield k

    def get_10x_lr_params(self):
        for mod in (self.layer5, self.layer6):
            for p in mod.parameters():
                yield p

    def optim_parameters(self, args):
        return [{'params': self.get_1x_lr_params_NOscale(), 'lr': args.learning_rate},
                {'params': self.get_10x_lr_params(), 'lr': 10 * args.learning_rate}]

    def _arena_segments(self):
        """(params, lr_group, multiplicity) ranges in first-appearance order."""
        counts, order = {}, []
        for p in self.get_1x_lr_params_NOscale():
            if id(p) not in counts:
                order.append(p)
            counts[id(p)] = counts.get(id(p), 0) + 1
        segs = []
        for mult in sorted(set(counts.values())):
            segs.append(([p for p in order if counts[id(p)] == mult], 0, mult))
        segs.append((list(self.get_10x_lr_params()), 1, 1))
        return segs

    # -- gradient buckets (data parallel) -----------------------------------------------
    def _bwd_units(self):
        """The generator backward's weight-gradient units in the order the engine finishes
        them (engine._DeeplabMultiFn.backward): layer6, layer4 blocks last to first, layer5,
        layer3 .. layer1 blocks last to first, the stem.  [(name, arena param indices)]."""
        A = self._arena

        def idx(*mods):
            return A.index_of([p for m in mods for p in m.parameters() if p.requires_grad])

        units = [("layer6", idx(self.layer6))]
        units += [(f"layer4.{i}", idx(self.layer4[i])) for i in reversed(range(len(self.layer4)))]
        units.append(("layer5", idx(self.layer5)))
        blocks = [(f"layer{li}.{i}", b) for li, layer in ((1, self.layer1), (2, self.layer2),
                                                          (3, self.layer3)) for i, b in enumerate(layer)]
        units += [(nm, idx(b)) for nm, b in reversed(blocks)]
        units.append(("stem", idx(self.conv1, self.bn1)))
        return units

    def _grad_buckets(self, bucket_bytes):
        """Split the gradient arena into all-reduce buckets that complete in backward order.

        Consecutive backward units are grouped until a bucket holds >= ``bucket_bytes``; a
        bucket is ready once the engine has launched the weight gradients of its last unit.
        Returns [(last_unit_ordinal, [(start, end), ...])] with each bucket's arena element
        ranges coalesced into contiguous runs (block convs, downsample convs and the 10x
        classifier sit in different arena segments, so a bucket spans 1-3 runs).  The runs of
        all buckets tile the arena exactly once (padding between parameters included)."""
        A = self._arena
        ends = A.offsets[1:] + [A.numel]
        units = self._bwd_units()
        seen = set()
        buckets, cur, cur_bytes = [], [], 0
        for ordinal, (_name, ids) in enumerate(units):
            ids = [i for i in ids if i not in seen]
            seen.update(ids)
            cur += ids
            cur_bytes += sum(4 * (ends[i] - A.offsets[i]) for i in ids)
            if cur and (cur_bytes >= bucket_bytes or ordinal == len(units) - 1):
                buckets.append((ordinal, cur))
                cur, cur_bytes = [], 0
        assert len(seen) == len(A.params), "every trainable parameter belongs to one unit"
        out = []
        for ordinal, ids in buckets:
            runs = []
            for i in sorted(ids, key=lambda i: A.offsets[i]):
                s, e = A.offsets[i], ends[i]
                if runs and runs[-1][1] == s:
                    runs[-1][1] = e
                else:
                    runs.append([s, e])
            out.append((ordinal, [tuple(r) for r in runs]))
        return out

    # -- arena --------------------------------------------------------------------------
    def _apply(self, fn, *args, **kwargs):
        self._arena_valid = False
        return super()._apply(fn, *args, **kwargs)

    def _ensure_arena(self, device):
        if self._arena_valid and self._arena is not None and self._arena.device == device:
            return
        self._arena = ParamArena(self._arena_segments(), device)
        A = self._arena

        def trainable(*mods):
            return A.index_of([p for m in mods for p in m.parameters() if p.requires_grad])

        self._pidx = {
            "trunk": trainable(self.conv1, self.layer1, self.layer2, self.layer3),
            "layer4": trainable(self.layer4),
            "layer5": trainable(self.layer5),
            "layer6": trainable(self.layer6),
        }
        bns = [m for m in self.modules() if isinstance(m, BatchNorm2d)]
        counter = torch.stack([bn.num_batches_tracked.detach().to(device) for bn in bns])
        for i, bn in enumerate(bns):
            bn.num_batches_tracked = counter[i]
        for bn in bns:
            for name in ("weight", "bias"):
                p = getattr(bn, name)
                if p.device != device:
                    p.data = p.data.to(device)
            for name in ("running_mean", "running_var"):
                setattr(bn, name, getattr(bn, name).to(device))
        self._bn_counter = counter
        self._anchors = {
            True: torch.empty(0, device=device, requires_grad=True),
            False: torch.empty(0, device=device, requires_grad=False),
        }
        self._arena_valid = True

    @property
    def arena(self) -> ParamArena:
        return self._arena

    # (the trainer's single-level step asks for the second head only)
    second_head_only_ok = True

    def forward(self, x, input_size=None, warper=None, first_head=True):
        """``first_head=False``: the layer5 head is not computed and its output is None — for
        callers that discard it (the single-level step's ``_, pred2 = model(...)``,
        train_gta2cityscapes_multi.py:405 / :421): pred2 is the same bit for bit."""
        if input_size is None:
            input_size = (x.shape[3], x.shape[2])
        x1_up, x2_up = engine.deeplab_multi_forward(self, x, input_size, first_head=first_head)
        if warper is not None:   # :190-192: both upsampled heads warped by the same field
            x1_up, x2_up = engine.grid_warp(warper, x1_up, x2_up)
        return x1_up, x2_up

    @staticmethod
    def warp(input, warper):
        """ResNetMulti.warp (model/deeplab_multi.py:238-255) on the HIP engine."""
        return engine.grid_warp(warper, None, input)[1]


def DeeplabMulti(num_classes=21):
    return ResNetMulti(Bottleneck, [3, 4, 23, 3], num_classes)
