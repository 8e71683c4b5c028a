"""TEST INFRASTRUCTURE ONLY — functional CPU restatement of the fork's Warper and its warp.

Stock PyTorch CPU ops over name->tensor dicts keyed like the reference's ``Warper().state_dict()``.
The numerical checker for the HIP warper engine (tests/, never the product path).  Pinned by
tests/golden/warper_goldens.npz, which gen_warper_golden.py captured from the reference's own
``model/warper.py`` / ``ResNetMulti.warp``.

Restated reference code (file:line in /root/reference), default ``Warper()`` configuration
(norm='Batch', warp_channels=2, num_layers=8, use_dropout=False, transpose=False):
  EncoderInput (4x4/2 conv, no bias)                 model/custom_layers.py:72-80
  DownConvolution (LeakyReLU(0.2, inplace) -> 4x4/2 conv -> BN)  :83-96
  EncoderOutput (LeakyReLU -> 4x4/2 conv)            :99-109
  DecoderInput / UpConvolution, non-transpose (ReLU(inplace) -> Upsample x2 bilinear
    align_corners=False -> 3x3 conv -> BN)           :117-139, :142-168
  DecoderOutput (ReLU -> Upsample x2 -> 3x3 conv + bias)                   :171-188
  SkipConnectionEncode.forward (skips reversed)      model/warper.py:36-64
  SkipConnectionDecode.forward (cat(skip, out))      model/warper.py:98-144
  Warper.__init__ / forward                          model/warper.py:216-267
  ResNetMulti.warp (tanh + linspace grid, clamp, grid_sample)  model/deeplab_multi.py:238-255
  source-only iteration                              train_gta2cityscapes_multi.py:259-286

The in-place LeakyReLU of each DownConvolution / EncoderOutput overwrites the previous
module's output, which SkipConnectionEncode has already stored as a skip connection: every
skip the decoder concatenates is therefore the LeakyReLU'd activation.  Likewise the
DecoderInput's in-place ReLU turns ``warp_list[0]`` (the clone of the latent) into relu(latent),
and the DecoderOutput's turns the last entry into relu(BN output).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .reference_torch import BN_EPS, BN_MOMENTUM

ENC_CH = (3, 64, 128, 256, 512, 512, 512, 512)        # down_list 0..6 outputs: ENC_CH[1..7]
DEC_IO = ((512, 512), (1024, 512), (1024, 512), (1024, 512), (1024, 256), (512, 128), (256, 64))
LEAKY = 0.2


def warper_specs(num_layers=8, warp_channels=2):
    """[(state_dict key, shape, kind)] of ``Warper()`` in registration order."""
    out = []
    for i in range(num_layers - 2 - 3):
        for sub in ("input", "one_one.1"):
            out.append((f"connection.one_one_list.{i}.{sub}.weight", (warp_channels, 512, 1, 1), "conv"))
            out.append((f"connection.one_one_list.{i}.{sub}.bias", (warp_channels,), "bias"))

    def bn(key, c):
        out.extend([(key + ".weight", (c,), "bn_w"), (key + ".bias", (c,), "bn_b"),
                    (key + ".running_mean", (c,), "bn_rm"), (key + ".running_var", (c,), "bn_rv"),
                    (key + ".num_batches_tracked", (), "bn_n")])

    out.append(("encoder_d.down_list.0.input.weight", (64, 3, 4, 4), "conv"))
    for k in range(1, 7):
        pre = f"encoder_d.down_list.{k}.block.1."
        out.append((pre + "l.weight", (ENC_CH[k + 1], ENC_CH[k], 4, 4), "conv"))
        bn(pre + "norm", ENC_CH[k + 1])
    out.append(("encoder_d.out.down.1.weight", (512, 512, 4, 4), "conv"))
    for i, (ci, co) in enumerate(DEC_IO):
        pre = f"decoder_d.up_list.{i}.block.2."
        out.append((pre + "l.weight", (co, ci, 3, 3), "conv"))
        bn(pre + "norm", co)
    out.append(("decoder_d.up_list.7.output.2.weight", (2, 64, 3, 3), "conv"))
    out.append(("decoder_d.up_list.7.output.2.bias", (2,), "bias"))
    return out


def warper_trainable(key):
    return not (".running_" in key or key.endswith("num_batches_tracked"))


def _bn(x, P, key, train):
    if train:
        P[key + ".num_batches_tracked"] += 1
    return F.batch_norm(x, P[key + ".running_mean"], P[key + ".running_var"], P[key + ".weight"],
                        P[key + ".bias"], train, BN_MOMENTUM, BN_EPS)


def _up2(x):
    # nn.Upsample(scale_factor=2, mode='bilinear'): align_corners defaults to False
    return F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)


def warper_forward(P, x, train=True):
    """Warper.forward(pose) -> (warp_output [N,2,H,W], warp_list of 8 tensors)."""
    out = F.conv2d(x, P["encoder_d.down_list.0.input.weight"], None, 2, 1)
    skips = [out]
    for k in range(1, 7):
        pre = f"encoder_d.down_list.{k}.block.1."
        out = F.leaky_relu(out, LEAKY)
        skips[-1] = out                      # the in-place LeakyReLU rewrites the stored skip
        out = _bn(F.conv2d(out, P[pre + "l.weight"], None, 2, 1), P, pre + "norm", train)
        skips.append(out)
    out = F.leaky_relu(out, LEAKY)
    skips[-1] = out
    latent = F.conv2d(out, P["encoder_d.out.down.1.weight"], None, 2, 1)
    skips.reverse()
    out = F.relu(latent)                     # DecoderInput's ReLU(True) on the clone in out_list
    out_list = [out]
    for i in range(len(DEC_IO)):
        if i != 0:
            out = torch.cat((skips[i - 1], out), 1)
        pre = f"decoder_d.up_list.{i}.block.2."
        out = _bn(F.conv2d(_up2(F.relu(out)), P[pre + "l.weight"], None, 1, 1), P, pre + "norm", train)
        out_list.append(out)
    out = F.relu(out)                        # DecoderOutput's ReLU(True): rewrites out_list[-1]
    out_list[-1] = out
    flow = F.conv2d(_up2(out), P["decoder_d.up_list.7.output.2.weight"],
                    P["decoder_d.up_list.7.output.2.bias"], 1, 1)
    return flow, out_list


def base_grid(h, w):
    """np.meshgrid(linspace(-1,1,W), linspace(-1,1,H)) stacked on the last axis, as float32
    (``torch.Tensor(xs)``): [..., 0] = x, [..., 1] = y."""
    xs = np.meshgrid(np.linspace(-1, 1, w), np.linspace(-1, 1, h))
    return torch.from_numpy(np.stack(xs, 2).astype(np.float32))


def warp(inp, flow):
    """ResNetMulti.warp(input, warper): only the LAST channel pair of the warper output is
    used (the loop overwrites ``sampler``); grid_sample with its defaults (bilinear, zeros,
    align_corners=False)."""
    n, c, h, w = inp.shape
    base = base_grid(h, w).unsqueeze(0).to(inp.dtype)
    sampler = None
    for i in range(flow.shape[1] // 2):
        sampler = (torch.tanh(flow[:, i * 2:(i + 1) * 2]).permute(0, 2, 3, 1) + base).clamp(-1, 1)
    return F.grid_sample(inp, sampler, mode="bilinear", padding_mode="zeros", align_corners=False)


def source_only_step(G, W, opt, cfg, i_iter, batches, bn_train=True):
    """One iteration of train_gta2cityscapes_multi.py:259-286 (SOURCE_ONLY, warper on).

    G / W: parameter dicts of DeeplabMulti / Warper; opt: the SGD of
    ``reference_torch.make_optimizers`` (the reference's ``optim_parameters`` groups).  The
    warper's parameters are never stepped (no optimiser holds them, :244); their gradients
    only accumulate.  The warper runs in train mode (:218).  Returns {"loss_seg2": value}.
    """
    from . import reference_torch as R
    c = dict(R.DEFAULT_CFG)
    c.update(cfg)
    opt.zero_grad()
    lr = R.lr_poly(c["learning_rate"], i_iter, c["num_steps"], c["power"])
    opt.param_groups[0]["lr"], opt.param_groups[1]["lr"] = lr, lr * 10
    n_sub = c["iter_size"]
    total = 0.0
    for images, labels in batches:
        flow, _ = warper_forward(W, images, train=True)
        _, pred2 = R.g_forward(G, images, c["input_size"], bn_train)
        pred2 = warp(pred2, flow)
        loss_seg2 = F.cross_entropy(pred2, labels, ignore_index=255)
        (loss_seg2 / n_sub).backward()
        total += loss_seg2.item() / n_sub
    opt.step()
    return {"loss_seg2": total}
