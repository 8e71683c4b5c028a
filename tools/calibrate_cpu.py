#!/usr/bin/env python3
"""Calibrate bench.py's CPU baseline (the oracle restatement) against the REFERENCE modules.

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu.py [--threads 8] [--reps 2]

Runs in the build container only (the reference cannot travel to the GPU box).  Times, on the
same host cores and inputs, (1) config c1 — DeeplabMulti(19) forward on 1x3x321x321 +
CrossEntropy2d — with /root/reference/model/deeplab_multi.py + utils/loss.py and with
oracle/reference_torch.py, and (2) one single-level adversarial step at batch 1, 1024x512 (the
c2 shape bench.py's ``cpu_baseline`` times) with the reference modules composed as
train_gta2cityscapes_multi.py:379-464 and with ``oracle_step``.  SURVEY §8(d) asks the
restatement to match the reference within +-10 %.  Writes profiles/<round>/cpu_calibration.json
(each round's run in its own directory: profiles/r1/, r4/, r5/ ...), with every rep's time and
the spread of the interleaved pairs' ratios, not only the best-of ratio.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from oracle import reference_torch as R  # noqa: E402


def best_of_pair(fa, fb, reps):
    """every time of fa and of fb over ``reps`` interleaved repetitions (after one warm-up each):
    alternating keeps allocator / oneDNN-cache / thermal drift from favouring either side (run
    back to back, the same pair measured anywhere from -12 % to +16 % apart)."""
    fa()
    fb()
    ta, tb = [], []
    for _ in range(reps):
        for f, ts in ((fa, ta), (fb, tb)):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
    return ta, tb


def record(out, name, ta, tb):
    """best-of times, their ratio, and the spread: every rep's time and the ratio of each
    interleaved pair (port / reference), min / median / max."""
    out[f"{name}_reference_s"], out[f"{name}_port_s"] = min(ta), min(tb)
    out[f"{name}_port_over_reference"] = min(tb) / min(ta)
    out[f"{name}_reference_reps_s"], out[f"{name}_port_reps_s"] = ta, tb
    pairs = sorted(b / a for a, b in zip(ta, tb))
    out[f"{name}_pair_ratios"] = pairs
    out[f"{name}_pair_ratio_min_median_max"] = [pairs[0], float(np.median(pairs)), pairs[-1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--round", default="r5", help="writes profiles/<round>/cpu_calibration.json")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    from gen_golden import load_ref, state_to_torch
    DeeplabMulti, FCDiscriminator, CrossEntropy2d = load_ref()
    warnings.simplefilter("ignore")
    out = {"threads": args.threads, "torch": torch.__version__}

    # ---- c1: forward + CrossEntropy2d, fp32 -----------------------------------------------
    x1 = torch.from_numpy(R.det_images((1, 3, 321, 321), 5)).float()
    l1 = torch.from_numpy(R.det_labels((1, 321, 321), 6))
    g = DeeplabMulti(num_classes=19)
    g.load_state_dict({k: v.float() if v.dtype.is_floating_point else v
                       for k, v in state_to_torch(R.det_state(R.g_specs(), 1338)).items()})
    g.train()
    ce = CrossEntropy2d()
    G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=torch.float32, trainable=R.g_trainable)

    def ref_c1():
        with torch.no_grad():
            _, p2 = g(x1, (321, 321))
            ce(p2, l1)

    def port_c1():
        with torch.no_grad():
            _, p2 = R.g_forward(G, x1, (321, 321), train=True)
            R.cross_entropy2d(p2, l1)

    record(out, "c1", *best_of_pair(ref_c1, port_c1, args.reps))

    # ---- c2 shape, batch 1: one single-level step ------------------------------------------
    xs = torch.from_numpy(R.det_images((1, 3, 512, 1024), 1)).float()
    lab = torch.from_numpy(R.det_labels((1, 512, 1024), 2))
    xt = torch.from_numpy(R.det_images((1, 3, 512, 1024), 3)).float()
    d2 = FCDiscriminator(num_classes=19)
    d2.load_state_dict({k: v.float() for k, v in state_to_torch(R.det_state(R.d_specs(), 2002)).items()})

    class Args:
        learning_rate = 2.5e-4

    opt = torch.optim.SGD(g.optim_parameters(Args), lr=2.5e-4, momentum=0.9, weight_decay=5e-4)
    od2 = torch.optim.Adam(d2.parameters(), lr=1e-4, betas=(0.9, 0.99))
    bce = torch.nn.BCEWithLogitsLoss()
    seg = torch.nn.CrossEntropyLoss(ignore_index=255)

    def ref_step():   # train_gta2cityscapes_multi.py:379-464 with the reference modules
        opt.zero_grad()
        od2.zero_grad()
        for p in d2.parameters():
            p.requires_grad = False
        _, pred2 = g(xs, (1024, 512))
        seg(pred2, lab).backward()
        _, pt2 = g(xt, (1024, 512))
        o = d2(F.softmax(pt2, dim=1))
        (0.001 * bce(o, torch.zeros_like(o))).backward()
        for p in d2.parameters():
            p.requires_grad = True
        o = d2(F.softmax(pred2.detach(), dim=1))
        (bce(o, torch.zeros_like(o)) / 2).backward()
        o = d2(F.softmax(pt2.detach(), dim=1))
        (bce(o, torch.ones_like(o)) / 2).backward()
        opt.step()
        od2.step()

    Gp = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=torch.float32, trainable=R.g_trainable)
    D2p = R.to_torch(R.det_state(R.d_specs(), 2002), dtype=torch.float32, trainable=lambda k: True)
    cfg = dict(level="single-level", gan="Vanilla", input_size=(1024, 512), input_size_target=(1024, 512))
    opts = R.make_optimizers(Gp, None, D2p, R.DEFAULT_CFG | cfg)

    def port_step():
        R.oracle_step(Gp, None, D2p, opts, cfg, 0, [(xs, lab, xt)])

    record(out, "c2b1_step", *best_of_pair(ref_step, port_step, args.reps))
    out["reps"] = args.reps
    path = os.path.join(REPO, "profiles", args.round, "cpu_calibration.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
