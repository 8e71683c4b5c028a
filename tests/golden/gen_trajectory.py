"""Full-resolution loss trajectories of the REFERENCE modules (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_trajectory.py [--quick]

Runs the reference's own DeeplabMulti / FCDiscriminator (imported read-only from
/root/reference) in fp32 on the CPU — the reference's dtype — from the deterministic
``oracle.reference_torch.det_state`` weights, for 5 iterations of the adversarial step on ONE
fixed synthetic batch (as bench.py does), at BASELINE's full geometries:

  c2: single-level, Vanilla (BCE), batch 1, source and target 1024x512
      (train_gta2cityscapes_multi.py:385-461), train-mode BN and eval-mode BN;
  c3: multi-level, Vanilla, batch 1, source 1280x720, target 1024x512 (:578-679, the target
      upsampled to input_size_target), train-mode BN.

Each trajectory is run twice, on 8 and on 3 CPU threads: the two runs differ only in fp32
summation order, so their distance is the reference's own numerical spread, against which
tests/test_fullres_gpu.py bounds the HIP engine's trajectory.  The fixture holds only the
per-iteration loss values (what the reference script prints, train:699-703).
"""
from __future__ import annotations

import argparse
import os
import sys
import time
import warnings

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from oracle import reference_torch as R  # noqa: E402
from gen_golden import D1_SEED, D2_SEED, G_SEED, load_ref  # noqa: E402

OUT = os.path.join(HERE, "trajectory_goldens.npz")
ITERS = 5
# name: (level, src (W, H), tgt (W, H), bn_train)
RUNS = {
    "c2_train": ("single-level", (1024, 512), (1024, 512), True),
    "c2_eval": ("single-level", (1024, 512), (1024, 512), False),
    "c3_train": ("multi-level", (1280, 720), (1024, 512), True),
}
LOSS_NAMES = {"single-level": ["loss_seg2", "loss_adv_target2", "loss_D2"],
              "multi-level": ["loss_seg1", "loss_seg2", "loss_adv_target1", "loss_adv_target2",
                              "loss_D1", "loss_D2"]}


def batch(src, tgt):
    """Fixed synthetic batch (seeds shared with tests/test_fullres_gpu.py)."""
    xs = torch.from_numpy(R.det_images((1, 3, src[1], src[0]), 11)).float()
    lab = torch.from_numpy(R.det_labels((1, src[1], src[0]), 12))
    xt = torch.from_numpy(R.det_images((1, 3, tgt[1], tgt[0]), 13)).float()
    return xs, lab, xt


def run(name, threads, iters):
    DeeplabMulti, FCDiscriminator, _ = load_ref()
    level, src, tgt, bn_train = RUNS[name]
    torch.set_num_threads(threads)

    def sd(specs, seed):
        return {k: torch.from_numpy(v.copy()).float() if v.dtype != np.int64 else torch.from_numpy(v.copy())
                for k, v in R.det_state(specs, seed).items()}

    g = DeeplabMulti(num_classes=19)
    g.load_state_dict(sd(R.g_specs(), G_SEED))
    d1 = FCDiscriminator(num_classes=19)
    d1.load_state_dict(sd(R.d_specs(), D1_SEED))
    d2 = FCDiscriminator(num_classes=19)
    d2.load_state_dict(sd(R.d_specs(), D2_SEED))
    g.train(bn_train)

    class Args:
        learning_rate = 2.5e-4

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        opt = torch.optim.SGD(g.optim_parameters(Args), lr=2.5e-4, momentum=0.9, weight_decay=5e-4,
                              foreach=False)
    od1 = torch.optim.Adam(d1.parameters(), lr=1e-4, betas=(0.9, 0.99), foreach=False)
    od2 = torch.optim.Adam(d2.parameters(), lr=1e-4, betas=(0.9, 0.99), foreach=False)
    bce = torch.nn.BCEWithLogitsLoss()
    seg = torch.nn.CrossEntropyLoss(ignore_index=255)
    xs, lab, xt = batch(src, tgt)
    out = []
    for it in range(iters):
        t0 = time.time()
        opt.zero_grad()
        lr = R.lr_poly(2.5e-4, it, 250000, 0.9)
        opt.param_groups[0]["lr"], opt.param_groups[1]["lr"] = lr, 10 * lr
        for o in (od1, od2):
            o.zero_grad()
            o.param_groups[0]["lr"] = R.lr_poly(1e-4, it, 250000, 0.9)
        if level == "single-level":   # train:385-461 (warper off)
            for p in d2.parameters():
                p.requires_grad = False
            _, p2 = g(xs, src)
            ls2 = seg(p2, lab)
            ls2.backward()
            _, pt2 = g(xt, src)       # :421 upsamples the target to input_size
            o2 = d2(F.softmax(pt2, dim=1))
            la2 = bce(o2, torch.zeros_like(o2))
            (0.001 * la2).backward()
            for p in d2.parameters():
                p.requires_grad = True
            ld = 0.0
            for q, lb in ((p2.detach(), 0.0), (pt2.detach(), 1.0)):
                o = d2(F.softmax(q, dim=1))
                l_ = bce(o, torch.full_like(o, lb)) / 2
                l_.backward()
                ld += l_.item()
            vals = [ls2.item(), la2.item(), ld]
        else:                         # :578-679, target -> input_size_target
            for d in (d1, d2):
                for p in d.parameters():
                    p.requires_grad = False
            p1, p2 = g(xs, src)
            ls1, ls2 = seg(p1, lab), seg(p2, lab)
            (ls2 + 0.1 * ls1).backward()
            pt1, pt2 = g(xt, tgt)
            o1, o2 = d1(F.softmax(pt1, dim=1)), d2(F.softmax(pt2, dim=1))
            la1, la2 = bce(o1, torch.zeros_like(o1)), bce(o2, torch.zeros_like(o2))
            (0.0002 * la1 + 0.001 * la2).backward()
            for d in (d1, d2):
                for p in d.parameters():
                    p.requires_grad = True
            ld1 = ld2 = 0.0
            for (q1, q2), lb in (((p1.detach(), p2.detach()), 0.0), ((pt1.detach(), pt2.detach()), 1.0)):
                o1, o2 = d1(F.softmax(q1, dim=1)), d2(F.softmax(q2, dim=1))
                a, b = bce(o1, torch.full_like(o1, lb)) / 2, bce(o2, torch.full_like(o2, lb)) / 2
                a.backward()
                b.backward()
                ld1 += a.item()
                ld2 += b.item()
            vals = [ls1.item(), ls2.item(), la1.item(), la2.item(), ld1, ld2]
        opt.step()
        od1.step()
        od2.step()
        out.append(vals)
        print(f"{name} threads={threads} iter {it}: " +
              " ".join(f"{k}={v:.5f}" for k, v in zip(LOSS_NAMES[level], vals)) + f"  ({time.time() - t0:.1f} s)",
              flush=True)
    return np.array(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="2 iterations, one thread count (smoke)")
    ap.add_argument("--only", default=None, help="comma-separated run names")
    args = ap.parse_args()
    iters = 2 if args.quick else ITERS
    names = args.only.split(",") if args.only else list(RUNS)
    gold = dict(np.load(OUT)) if os.path.exists(OUT) and args.only else {}
    for name in names:
        for threads in ((8,) if args.quick else (8, 3)):
            gold[f"{name}/threads{threads}"] = run(name, threads, iters)
        gold[f"{name}/names"] = np.array(LOSS_NAMES[RUNS[name][0]])
    gold["meta"] = np.array(repr(dict(iters=iters, g_seed=G_SEED, d1_seed=D1_SEED, d2_seed=D2_SEED,
                                      runs=RUNS, torch=torch.__version__, dtype="float32")))
    np.savez_compressed(OUT, **gold)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
