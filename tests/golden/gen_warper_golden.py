"""Capture golden vectors of the fork's Warper from the REFERENCE code (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_warper_golden.py

Imports /root/reference/model/{warper,deeplab_multi}.py (read-only, no bytecode written),
loads deterministic fp64 weights (``oracle.reference_warper.warper_specs`` +
``oracle.reference_torch.det_state``) and records into tests/golden/warper_goldens.npz:

  1. ``Warper().train()`` forward on a 2x3x256x256 batch: the flow (every 4th pixel) and
     checksums of the full flow and of each ``warp_list`` entry, BN running statistics; the
     backward of <flow, R>: per-parameter gradient norms and two full gradients;
  2. ``ResNetMulti.warp(input, warper)`` (deeplab_multi.py:238-255) on small inputs, moderate
     and saturating flows (inputs regenerated from their PCG64 seeds by the tests): outputs
     and the gradients of <out, R> w.r.t. input and flow;
  3. two iterations of the SOURCE_ONLY step with the warper on
     (train_gta2cityscapes_multi.py:259-286): reference DeeplabMulti + Warper, the reference's
     own ``optim_parameters`` SGD, nn.CrossEntropyLoss(ignore_index=255): losses, parameter
     checksums after the steps, accumulated warper gradient norms.

``ResNetMulti.warp`` moves a zeros tensor to the GPU with an unconditional ``.cuda()`` (whose
value it then discards); this container has no GPU, so ``torch.Tensor.cuda`` is replaced by the
identity while capturing.  Only inputs/outputs are stored — no reference source.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import reference_torch as R  # noqa: E402
from oracle import reference_warper as RW  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(HERE, "warper_goldens.npz")

W_SEED, G_SEED = 3001, 1338
W_CONV_STD = 0.02
IMG_SHAPE = (2, 3, 256, 256)
WARP_IN, WARP_FLOW = (2, 19, 16, 24), (2, 2, 16, 24)


def load_ref():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from model.warper import Warper  # noqa: E402
    from model.deeplab_multi import DeeplabMulti, ResNetMulti  # noqa: E402
    return Warper, DeeplabMulti, ResNetMulti


def to_ref(sd):
    return {k: torch.from_numpy(v.copy()).double() if v.dtype != np.int64 else torch.from_numpy(v.copy())
            for k, v in sd.items()}


def det_normal(shape, seed, scale=1.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(scale * rng.standard_normal(shape))


def main():
    Warper, DeeplabMulti, ResNetMulti = load_ref()
    torch.set_num_threads(8)
    torch.Tensor.cuda = lambda self, *a, **k: self     # see module docstring
    gold = {}
    x = torch.from_numpy(R.det_images(IMG_SHAPE, 21))

    # ---- 1. Warper forward / backward ------------------------------------------------------
    w = Warper().double()
    w.load_state_dict(to_ref(R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD)))
    w.train()
    flow, warp_list = w(x)
    gold["warper/flow_s4"] = flow.detach()[:, :, ::4, ::4].numpy()
    gold["warper/flow_sum"] = np.array(flow.detach().sum().item())
    gold["warper/flow_norm"] = np.array(flow.detach().norm().item())
    for i, t in enumerate(warp_list):
        gold[f"warper/list{i}_shape"] = np.array(t.shape)
        gold[f"warper/list{i}_sum"] = np.array(t.detach().sum().item())
        gold[f"warper/list{i}_norm"] = np.array(t.detach().norm().item())
    rw = det_normal(flow.shape, 22)
    (flow * rw).sum().backward()
    for k, p in w.named_parameters():
        if p.grad is not None:
            gold[f"warper/gradnorm/{k}"] = np.array(p.grad.norm().item())
    gold["warper/grad/encoder_d.down_list.0.input.weight"] = w.encoder_d.down_list[0].input.weight.grad.numpy()
    gold["warper/grad/decoder_d.up_list.7.output.2.weight"] = w.decoder_d.up_list[7].output[2].weight.grad.numpy()
    gold["warper/grad/decoder_d.up_list.7.output.2.bias"] = w.decoder_d.up_list[7].output[2].bias.grad.numpy()
    for k, v in w.state_dict().items():
        if "running" in k:
            gold[f"warper/sum/{k}"] = np.array(v.sum().item())

    # ---- 2. ResNetMulti.warp ----------------------------------------------------------------
    for tag, scale in (("mod", 0.8), ("sat", 6.0)):
        inp = det_normal(WARP_IN, 23).requires_grad_(True)
        fl = det_normal(WARP_FLOW, 24, scale).requires_grad_(True)
        out = ResNetMulti.warp(inp, fl)
        r = det_normal(out.shape, 25)
        (out * r).sum().backward()
        gold[f"warp_{tag}/out"] = out.detach().numpy()
        gold[f"warp_{tag}/d_input"] = inp.grad.numpy()
        gold[f"warp_{tag}/d_flow"] = fl.grad.numpy()

    # ---- 3. SOURCE_ONLY step with the warper -----------------------------------------------
    g = DeeplabMulti(num_classes=19).double()
    g.load_state_dict(to_ref(R.det_state(R.g_specs(), G_SEED)))
    w = Warper().double()
    w.load_state_dict(to_ref(R.det_state(RW.warper_specs(), W_SEED, conv_std=W_CONV_STD)))
    g.train()
    w.train()
    cfg = R.DEFAULT_CFG

    class _A:
        learning_rate = cfg["learning_rate"]
    opt = torch.optim.SGD(g.optim_parameters(_A), lr=cfg["learning_rate"], momentum=cfg["momentum"],
                          weight_decay=cfg["weight_decay"])
    lab = torch.from_numpy(R.det_labels((IMG_SHAPE[0], IMG_SHAPE[2], IMG_SHAPE[3]), 26))
    seg_loss = torch.nn.CrossEntropyLoss(ignore_index=255)
    in_size = (IMG_SHAPE[3], IMG_SHAPE[2])
    for it in range(2):
        opt.zero_grad()
        lr = R.lr_poly(cfg["learning_rate"], it, cfg["num_steps"], cfg["power"])
        opt.param_groups[0]["lr"], opt.param_groups[1]["lr"] = lr, 10 * lr
        warper, _ = w(x)
        _, pred2 = g(x, in_size, warper)
        loss = seg_loss(pred2, lab)
        loss.backward()
        gold[f"source_only/loss_seg2/{it}"] = np.array(loss.item())
        opt.step()
    for k, v in g.state_dict().items():
        if v.dtype.is_floating_point and ("layer4.2" in k or "layer6" in k or k == "conv1.weight"):
            gold[f"source_only/sum/{k}"] = np.array(v.double().sum().item())
            gold[f"source_only/norm/{k}"] = np.array(v.double().norm().item())
    for k, p in w.named_parameters():
        if p.grad is not None:
            gold[f"source_only/warper_gradnorm/{k}"] = np.array(p.grad.norm().item())
    np.savez_compressed(OUT, **gold)
    print(f"wrote {OUT}: {len(gold)} arrays, {os.path.getsize(OUT) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
