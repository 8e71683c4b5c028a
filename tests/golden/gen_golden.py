"""Capture golden vectors from the REFERENCE modules (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Imports /root/reference/{model/deeplab_multi.py, model/discriminator.py, utils/loss.py}
(read-only; no bytecode written), loads deterministic fp64 weights from
``oracle.reference_torch.det_state`` into them, and records outputs, losses, gradient
norms and post-step parameter checksums into tests/golden/reference_goldens.npz.  The
step bodies follow train_gta2cityscapes_multi.py:379-464 (single-level) and :570-683
(multi-level) with the reference's own optimiser construction (optim_parameters, Adam).
Only inputs/outputs are stored — no reference source.
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import reference_torch as R  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(HERE, "reference_goldens.npz")

# Geometry of the captures (small enough for CPU fp64 in seconds).
G_SEED, D1_SEED, D2_SEED = 1338, 2001, 2002
SRC_SHAPE, TGT_SHAPE = (2, 3, 41, 57), (2, 3, 33, 49)


def load_ref():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from model.deeplab_multi import DeeplabMulti  # noqa: E402
    from model.discriminator import FCDiscriminator  # noqa: E402
    from utils.loss import CrossEntropy2d  # noqa: E402
    return DeeplabMulti, FCDiscriminator, CrossEntropy2d


def state_to_torch(sd):
    return {k: torch.from_numpy(v.copy()).double() if v.dtype != np.int64 else torch.from_numpy(v.copy())
            for k, v in sd.items()}


def build(DeeplabMulti, FCDiscriminator):
    g = DeeplabMulti(num_classes=19).double()
    g.load_state_dict(state_to_torch(R.det_state(R.g_specs(), G_SEED)))
    d1 = FCDiscriminator(num_classes=19).double()
    d1.load_state_dict(state_to_torch(R.det_state(R.d_specs(), D1_SEED)))
    d2 = FCDiscriminator(num_classes=19).double()
    d2.load_state_dict(state_to_torch(R.det_state(R.d_specs(), D2_SEED)))
    return g, d1, d2


def inputs():
    xs = torch.from_numpy(R.det_images(SRC_SHAPE, 11))
    lab = torch.from_numpy(R.det_labels((SRC_SHAPE[0], SRC_SHAPE[2], SRC_SHAPE[3]), 12))
    xt = torch.from_numpy(R.det_images(TGT_SHAPE, 13))
    return xs, lab, xt


def param_norms(model, prefix):
    out = {}
    for k, p in model.named_parameters():
        if p.grad is not None:
            out[f"{prefix}gradnorm/{k}"] = np.array(p.grad.norm().item())
    return out


def checksums(model, prefix):
    out = {}
    for k, v in model.state_dict().items():
        if v.dtype.is_floating_point:
            out[f"{prefix}sum/{k}"] = np.array(v.double().sum().item())
            out[f"{prefix}norm/{k}"] = np.array(v.double().norm().item())
        else:
            out[f"{prefix}int/{k}"] = np.array(int(v.item()))
    return out


def main():
    DeeplabMulti, FCDiscriminator, CrossEntropy2d = load_ref()
    torch.set_num_threads(8)
    gold = {}
    xs, lab, xt = inputs()
    in_size = (SRC_SHAPE[3], SRC_SHAPE[2])       # (W, H) — train:191-195
    in_size_t = (TGT_SHAPE[3], TGT_SHAPE[2])

    # ---- 1. forward (train-mode BN) + CrossEntropy2d + backward ----------------------
    g, d1, d2 = build(DeeplabMulti, FCDiscriminator)
    g.train()
    p1, p2 = g(xs, in_size)
    gold["fwd_train/pred1"] = p1.detach().numpy().astype(np.float32)
    gold["fwd_train/pred2"] = p2.detach().numpy().astype(np.float32)
    ce = CrossEntropy2d()
    l2 = ce(p2, lab)
    l_nn = torch.nn.CrossEntropyLoss(ignore_index=255)(p2, lab)
    gold["ce/crossentropy2d"] = np.array(l2.item())
    gold["ce/nn_crossentropy"] = np.array(l_nn.item())
    (l2 + 0.1 * ce(p1, lab)).backward()
    gold.update(param_norms(g, "bwd_train/"))
    gold["bwd_train/grad/conv1.weight"] = g.conv1.weight.grad.numpy()
    gold["bwd_train/grad/layer6.conv2d_list.0.bias"] = g.layer6.conv2d_list[0].bias.grad.numpy()
    gold.update({k: v for k, v in checksums(g, "fwd_train/").items() if "running" in k or "/int/" in k})

    # ---- 2. eval-mode forward ---------------------------------------------------------
    g, d1, d2 = build(DeeplabMulti, FCDiscriminator)
    g.eval()
    with torch.no_grad():
        e1, e2 = g(xs, in_size)
    gold["fwd_eval/pred1"] = e1.numpy().astype(np.float32)
    gold["fwd_eval/pred2"] = e2.numpy().astype(np.float32)

    # ---- 3. discriminator forward/backward + adversarial losses -------------------------
    sm = F.softmax(p2.detach(), dim=1).requires_grad_(True)
    dout = d1(sm)
    gold["d/out"] = dout.detach().numpy()
    bce = torch.nn.BCEWithLogitsLoss()(dout, torch.zeros_like(dout))
    mse = torch.nn.MSELoss()(dout, torch.ones_like(dout))
    gold["d/bce0"] = np.array(bce.item())
    gold["d/mse1"] = np.array(mse.item())
    (bce + mse).backward()
    gold["d/input_grad"] = sm.grad.numpy()
    gold.update(param_norms(d1, "d/"))

    # ---- 4. CrossEntropy2d edge cases ---------------------------------------------------
    rng = np.random.Generator(np.random.PCG64(99))
    logits = torch.from_numpy(rng.standard_normal((2, 19, 5, 7)))
    tl = torch.from_numpy(rng.integers(-1, 19, (2, 5, 7)).astype(np.int64))
    tl[0, 0, :3] = 255
    gold["ce_edge/logits_seed"] = np.array(99)
    gold["ce_edge/loss"] = np.array(CrossEntropy2d()(logits, tl).item())
    allign = torch.full((1, 4, 4), 255, dtype=torch.int64)
    gold["ce_edge/all_ignored_is_nan"] = np.array(
        bool(torch.isnan(CrossEntropy2d()(torch.from_numpy(rng.standard_normal((1, 19, 4, 4))), allign)).item()))

    # ---- 5. one full step, single-level and multi-level, Vanilla and LS ----------------
    class Args:
        learning_rate = 2.5e-4
        learning_rate_D = 1e-4

    for level, gan in (("single-level", "Vanilla"), ("multi-level", "LS")):
        g, d1, d2 = build(DeeplabMulti, FCDiscriminator)
        g.train()
        d1.train()
        d2.train()
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            opt = torch.optim.SGD(g.optim_parameters(Args), lr=2.5e-4, momentum=0.9,
                                  weight_decay=5e-4, foreach=False)
        od1 = torch.optim.Adam(d1.parameters(), lr=1e-4, betas=(0.9, 0.99), foreach=False)
        od2 = torch.optim.Adam(d2.parameters(), lr=1e-4, betas=(0.9, 0.99), foreach=False)
        bce_loss = torch.nn.BCEWithLogitsLoss() if gan == "Vanilla" else torch.nn.MSELoss()
        seg_loss = torch.nn.CrossEntropyLoss(ignore_index=255)
        pre = f"step_{level}_{gan}/"
        vals = {}
        for i_iter in range(2):  # two iterations: exercises momentum / Adam state
            opt.zero_grad()
            lr = R.lr_poly(2.5e-4, i_iter, 250000, 0.9)
            opt.param_groups[0]["lr"], opt.param_groups[1]["lr"] = lr, 10 * lr
            lrd = R.lr_poly(1e-4, i_iter, 250000, 0.9)
            for o in (od1, od2):
                o.zero_grad()
                o.param_groups[0]["lr"] = lrd
            if level == "single-level":
                for p in d2.parameters():
                    p.requires_grad = False
                _, pred2 = g(xs, in_size)
                ls2 = seg_loss(pred2, lab)
                ls2.backward()
                _, pt2 = g(xt, in_size)      # train:421 upsamples the target to input_size
                d_o = d2(F.softmax(pt2, dim=1))
                la2 = bce_loss(d_o, torch.zeros_like(d_o))
                (0.001 * la2).backward()
                for p in d2.parameters():
                    p.requires_grad = True
                d_o = d2(F.softmax(pred2.detach(), dim=1))
                ld_a = bce_loss(d_o, torch.zeros_like(d_o)) / 2
                ld_a.backward()
                d_o = d2(F.softmax(pt2.detach(), dim=1))
                ld_b = bce_loss(d_o, torch.ones_like(d_o)) / 2
                ld_b.backward()
                vals[i_iter] = [ls2.item(), la2.item(), ld_a.item() + ld_b.item()]
            else:
                for d in (d1, d2):
                    for p in d.parameters():
                        p.requires_grad = False
                pred1, pred2 = g(xs, in_size)
                ls1, ls2 = seg_loss(pred1, lab), seg_loss(pred2, lab)
                (ls2 + 0.1 * ls1).backward()
                pt1, pt2 = g(xt, in_size_t)  # resolved: target -> input_size_target
                o1, o2 = d1(F.softmax(pt1, dim=1)), d2(F.softmax(pt2, dim=1))
                la1 = bce_loss(o1, torch.zeros_like(o1))
                la2 = bce_loss(o2, torch.zeros_like(o2))
                (0.0002 * la1 + 0.001 * la2).backward()
                for d in (d1, d2):
                    for p in d.parameters():
                        p.requires_grad = True
                lds = []
                for (q1, q2), lb in (((pred1.detach(), pred2.detach()), 0.0),
                                     ((pt1.detach(), pt2.detach()), 1.0)):
                    o1, o2 = d1(F.softmax(q1, dim=1)), d2(F.softmax(q2, dim=1))
                    l1 = bce_loss(o1, torch.full_like(o1, lb)) / 2
                    l2b = bce_loss(o2, torch.full_like(o2, lb)) / 2
                    l1.backward()
                    l2b.backward()
                    lds += [l1.item(), l2b.item()]
                vals[i_iter] = [ls1.item(), ls2.item(), la1.item(), la2.item(),
                                lds[0] + lds[2], lds[1] + lds[3]]
            opt.step()
            od1.step()
            od2.step()
        for i_iter, v in vals.items():
            gold[pre + f"losses_iter{i_iter}"] = np.array(v)
        gold.update({pre + k: v for k, v in checksums(g, "G/").items()})
        gold.update({pre + k: v for k, v in checksums(d2, "D2/").items()})
        if level == "multi-level":
            gold.update({pre + k: v for k, v in checksums(d1, "D1/").items()})

    meta = dict(g_seed=G_SEED, d1_seed=D1_SEED, d2_seed=D2_SEED, src=SRC_SHAPE, tgt=TGT_SHAPE,
                torch=torch.__version__)
    gold["meta"] = np.array(repr(meta))
    np.savez_compressed(OUT, **gold)
    print(f"wrote {OUT}: {len(gold)} arrays, {os.path.getsize(OUT) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
