"""The fork's Warper (pix2pix-style U-Net that outputs a 2-channel warp field) on the HIP engine.

Drop-in for /root/reference/model/warper.py:216-267 with its building blocks from
model/custom_layers.py: same class names, constructor and forward signatures, module tree and
therefore the same ``state_dict()`` keys (``connection.one_one_list.*``,
``encoder_d.down_list.{0..6}.*``, ``encoder_d.out.down.1.weight``, ``decoder_d.up_list.{0..7}.*``),
and the same ``init_weights(net, 'xavier', 0.02)`` initialisation (:182-213).  The arithmetic
runs in ``adaptsegnet_amd.engine`` (``_WarperFn``); the ReLU / LeakyReLU / Upsample / Dropout
children are structural only (never called), as the reference's hold no parameters.

Supported configuration: the one the training script builds, ``Warper()`` (norm='Batch',
transpose=False, use_dropout=False, use_advanced=False; any ``num_layers`` >= 5 and
``warp_channels``).  The transpose-convolution, spectral / instance norm and dropout variants
are not used by the reference's scripts and raise ``NotImplementedError``.

Reference semantics kept (file:line):
  Connection (built, never called in forward)          model/warper.py:15-33
  SkipConnectionEncode / SkipConnectionDecode          :36-64, :98-144
  Warper.__init__ / forward / flip_warp                :216-267
  EncoderInput / DownConvolution / EncoderOutput       model/custom_layers.py:72-109
  DecoderInput / UpConvolution / DecoderOutput         :117-188
  OneOneConvolution / NaiveConvolution                 :25-33, :52-63
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
from torch.nn import init

from .. import engine
from .layers import BatchNorm2d, Conv2d, ParamArena


class NaiveConvolution(nn.Module):
    def __init__(self, in_ch, out_ch, w, s, p, bias, norm_layer):
        super().__init__()
        self.l = Conv2d(in_ch, out_ch, kernel_size=w, stride=s, padding=p, bias=bias)
        self.norm = norm_layer(out_ch)


class OneOneConvolution(nn.Module):
    def __init__(self, in_ch, out_ch, use_bias):
        super().__init__()
        self.input = Conv2d(in_ch, out_ch, kernel_size=1, stride=1, padding=0, bias=use_bias)
        self.one_one = nn.Sequential(nn.ReLU(True), Conv2d(in_ch, out_ch, kernel_size=1, stride=1, padding=0,
                                                           bias=use_bias))


class EncoderInput(nn.Module):
    def __init__(self, in_ch, out_ch, use_bias):
        super().__init__()
        self.input = Conv2d(in_ch, out_ch, kernel_size=4, stride=2, padding=1, bias=use_bias)


class DownConvolution(nn.Module):
    def __init__(self, in_ch, out_ch, use_bias, norm_layer):
        super().__init__()
        if norm_layer == "Spectral":
            raise NotImplementedError("Warper: spectral-norm blocks are not supported")
        self.block = nn.Sequential(nn.LeakyReLU(0.2, True),
                                   NaiveConvolution(in_ch, out_ch, w=4, s=2, p=1, bias=use_bias,
                                                    norm_layer=norm_layer))


class EncoderOutput(nn.Module):
    def __init__(self, in_ch, out_ch, use_bias):
        super().__init__()
        self.down = nn.Sequential(nn.LeakyReLU(0.2, True),
                                  Conv2d(in_ch, out_ch, kernel_size=4, stride=2, padding=1, bias=use_bias))


def _check_up(norm_layer, transpose):
    if transpose:
        raise NotImplementedError("Warper: transpose-convolution decoder (transpose=True) is not supported")
    if norm_layer == "Spectral":
        raise NotImplementedError("Warper: spectral-norm blocks are not supported")


class DecoderInput(nn.Module):
    def __init__(self, in_ch, out_ch, use_bias, norm_layer, use_transpose):
        super().__init__()
        _check_up(norm_layer, use_transpose)
        self.block = nn.Sequential(nn.ReLU(True), nn.Upsample(scale_factor=2, mode="bilinear"),
                                   NaiveConvolution(in_ch, out_ch, w=3, s=1, p=1, bias=use_bias,
                                                    norm_layer=norm_layer))


class UpConvolution(nn.Module):
    def __init__(self, in_ch, out_ch, use_bias, norm_layer, use_dropout, use_transpose):
        super().__init__()
        _check_up(norm_layer, use_transpose)
        if use_dropout:
            raise NotImplementedError("Warper: use_dropout=True is not supported")
        self.block = nn.Sequential(nn.ReLU(True), nn.Upsample(scale_factor=2, mode="bilinear"),
                                   NaiveConvolution(in_ch, out_ch, w=3, s=1, p=1, bias=use_bias,
                                                    norm_layer=norm_layer))
        self.use_dropout = use_dropout
        self.dropout = nn.Dropout(0.5)


class DecoderOutput(nn.Module):
    def __init__(self, in_ch, out_ch, use_transpose):
        super().__init__()
        _check_up(None, use_transpose)
        self.output = nn.Sequential(nn.ReLU(True), nn.Upsample(scale_factor=2, mode="bilinear"),
                                    Conv2d(in_ch, out_ch, kernel_size=3, stride=1, padding=1, bias=True))


def _batch_norm(c):
    return BatchNorm2d(c)


def _norm(norm_layer):
    if norm_layer != "Batch":
        raise NotImplementedError(f"Warper: norm {norm_layer!r} is not supported (only 'Batch')")
    return False, _batch_norm


class Connection(nn.Module):
    """Built by the reference but never called by Warper.forward (model/warper.py:15-33)."""

    def __init__(self, num_layers=6, warp_channels=2):
        super().__init__()
        self.num_layers = num_layers
        self.one_one_list = nn.ModuleList(
            [OneOneConvolution(512, warp_channels if warp_channels else 2 * 512, True)
             for _ in range(num_layers - 3)])


class SkipConnectionEncode(nn.Module):
    def __init__(self, norm_layer="Batch", out_channel=512, num_layers=8):
        super().__init__()
        self.use_bias, self.norm_layer = _norm(norm_layer)
        self.num_layers = num_layers
        down = [EncoderInput(3, 64, self.use_bias),
                DownConvolution(64, 128, self.use_bias, self.norm_layer),
                DownConvolution(128, 256, self.use_bias, self.norm_layer),
                DownConvolution(256, 512, self.use_bias, self.norm_layer)]
        down += [DownConvolution(512, 512, self.use_bias, self.norm_layer) for _ in range(num_layers - 5)]
        self.down_list = nn.ModuleList(down)
        self.out = EncoderOutput(512, out_channel, self.use_bias)


class SkipConnectionDecode(nn.Module):
    def __init__(self, norm_layer="Batch", out_channel=3, num_layers=8, use_dropout=False, transpose=True,
                 use_advanced=False):
        super().__init__()
        if use_advanced:
            raise NotImplementedError("Warper: use_advanced=True is not supported")
        self.use_bias, self.norm_layer = _norm(norm_layer)
        self.use_advanced = use_advanced
        self.num_layers = num_layers
        up = [DecoderInput(512, 512, self.use_bias, self.norm_layer, transpose)]
        up += [UpConvolution(1024, 512, self.use_bias, self.norm_layer, use_dropout, transpose)
               for _ in range(num_layers - 4)]
        up += [UpConvolution(1024, 256, self.use_bias, self.norm_layer, use_dropout, transpose),
               UpConvolution(512, 128, self.use_bias, self.norm_layer, use_dropout, transpose),
               UpConvolution(256, 64, self.use_bias, self.norm_layer, use_dropout, transpose),
               DecoderOutput(64, out_channel, transpose)]
        self.up_list = nn.ModuleList(up)


def init_weights(net, init_type="normal", init_gain=0.02):
    """model/warper.py:182-213: conv weights N(0, gain) / xavier / kaiming / orthogonal, biases 0;
    BatchNorm weights N(1, gain), biases 0."""
    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
            with torch.no_grad():
                if init_type == "normal":
                    init.normal_(m.weight, 0.0, init_gain)
                elif init_type == "xavier":
                    init.xavier_normal_(m.weight, gain=init_gain)
                elif init_type == "kaiming":
                    init.kaiming_normal_(m.weight, a=0, mode="fan_in")
                elif init_type == "orthogonal":
                    init.orthogonal_(m.weight, gain=init_gain)
                else:
                    raise NotImplementedError("initialization method [%s] is not implemented" % init_type)
                if getattr(m, "bias", None) is not None:
                    init.constant_(m.bias, 0.0)
        elif classname.find("BatchNorm2d") != -1:
            with torch.no_grad():
                init.normal_(m.weight, 1.0, init_gain)
                init.constant_(m.bias, 0.0)

    net.apply(init_func)
    return net


class Warper(nn.Module):
    def __init__(self, norm="Batch", warp_channels=2, num_layers=8, use_dropout=False, transpose=False,
                 warp_out=False, use_advanced=False):
        super().__init__()
        init_gain, init_type = 0.02, "xavier"
        driving_num_layers = num_layers - 1
        self.connection = init_weights(Connection(num_layers - 2, warp_channels), init_type, init_gain)
        self.encoder_d = init_weights(SkipConnectionEncode(norm, 512, num_layers), init_type, init_gain)
        self.decoder_d = init_weights(SkipConnectionDecode(norm, 2, driving_num_layers, use_dropout, transpose),
                                      init_type, init_gain)
        self._arena = None
        self._arena_valid = False

    # -- engine plumbing (as FCDiscriminator) ----------------------------------------------
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
        bns = [m for m in self.modules() if isinstance(m, BatchNorm2d)]
        counter = torch.stack([bn.num_batches_tracked.detach().to(device) for bn in bns])
        for i, bn in enumerate(bns):
            bn.num_batches_tracked = counter[i]
            for name in ("running_mean", "running_var"):
                setattr(bn, name, getattr(bn, name).to(device))
        self._bn_counter = counter
        self._arena_valid = True

    @property
    def arena(self) -> ParamArena:
        return self._arena

    def encoder_blocks(self):
        """[(conv, bn or None)] of down_list, then the EncoderOutput conv."""
        out = [(self.encoder_d.down_list[0].input, None)]
        out += [(m.block[1].l, m.block[1].norm) for m in self.encoder_d.down_list[1:]]
        return out, self.encoder_d.out.down[1]

    def decoder_blocks(self):
        """[(conv, bn)] of the NaiveConvolution blocks, then the DecoderOutput conv."""
        ups = self.decoder_d.up_list
        return [(m.block[2].l, m.block[2].norm) for m in ups[:-1]], ups[-1].output[2]

    @staticmethod
    def flip_warp(warp_list):
        """model/warper.py:243-261: a detached copy of each entry with its first channel negated
        (the reference builds the +-1 mask with size(-1) for both spatial dims, i.e. square maps)."""
        out = [0] * len(warp_list)
        for i, warper in enumerate(list(warp_list)):
            wc = warper.detach()
            ones = np.ones((1, wc.size(-1), wc.size(-1)))
            flipper = torch.tensor(np.concatenate((-ones, ones), 0), dtype=torch.float32, device=wc.device)
            out[i] = flipper.unsqueeze(0).repeat(wc.size(0), 1, 1, 1) * wc
        return out

    def forward(self, pose, warper_flip=False):
        """-> (warp_output [N,2,H,W], warp_list): the flow and the decoder's intermediate maps
        (``warp_list[0]`` = relu(latent), then each decoder block's BatchNorm output), as
        SkipConnectionDecode.forward returns them.  The warp_list entries carry no gradient."""
        return engine.warper_forward(self, pose)
