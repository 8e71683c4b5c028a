#!/usr/bin/env python3
"""Per-shape cost of the fused BN backward sums (conv_dgrad(bnsum=...) + bn_bwd(sums=...)) against
the unfused chain (conv_dgrad + bn_bwd with its own reduction pass), alone on the GPU: for each
Bottleneck data gradient of the c2 step that feeds a BN+ReLU backward (conv3 -> bn2, conv2 -> bn1),
the data-gradient kernel, the BN backward and their sum, in microseconds.

    python tools/bnsum_bench.py [--batch 4] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from adaptsegnet_amd import kernels as K  # noqa: E402


def shapes(batch, H=512, W=1024):
    h, w = (H + 1) // 2, (W + 1) // 2
    h, w = (h + 1) // 2, (w + 1) // 2
    out = []
    for li, (planes, stride, dil) in enumerate(((64, 1, 1), (128, 2, 1), (256, 1, 2), (512, 1, 4)), 1):
        oh, ow = (h - 1) // stride + 1, (w - 1) // stride + 1
        out.append((f"l{li}.conv3->bn2", K.ConvGeom(planes, planes * 4, 1, 1), batch, oh, ow))
        out.append((f"l{li}.conv2->bn1", K.ConvGeom(planes, planes, 3, 3, 1, (dil,), (dil,)), batch, oh, ow))
        h, w = oh, ow
    return out


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    print(f"{'product':18s} {'tiles':>5s} {'dgrad':>8s} {'+sums':>8s} {'bn_bwd':>8s} {'bn_sums':>8s} "
          f"{'unfused':>8s} {'fused':>8s}")
    tot_u = tot_f = 0.0
    for name, g, n, h, w in shapes(args.batch):
        oh, ow = g.out_hw(h, w)
        c = g.cin
        dy = torch.randn(n, oh, ow, g.cout, device=dev)
        wt = torch.randn(g.cout, g.kh, g.kw, c, device=dev) * 0.05
        x = torch.randn(n, h, w, c, device=dev)
        bw, bb = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
        _, mean, invstd = K.bn_fwd_train(x, bw, bb, torch.zeros(c, device=dev), torch.ones(c, device=dev), 0.1, 1e-5)
        spec = K.BnSum(x, mean, invstd, bw, bb, K.BNSUM_RELU_X)
        dx = K.conv_dgrad(g, dy, n, h, w, [wt])
        _, sums = K.conv_dgrad(g, dy, n, h, w, [wt], bnsum=spec)
        nt = sums[1] if sums else 0
        t_d = timed(lambda: K.conv_dgrad(g, dy, n, h, w, [wt], out=dx), args.reps)
        t_ds = timed(lambda: K.conv_dgrad(g, dy, n, h, w, [wt], out=dx, bnsum=spec), args.reps)
        out = torch.empty_like(dx)
        t_b = timed(lambda: K.bn_bwd(dx, None, x, bw, mean, invstd, relu=True, dx=out, bias=bb), args.reps)
        t_bs = timed(lambda: K.bn_bwd(dx, None, x, bw, mean, invstd, relu=True, dx=out, bias=bb, sums=sums),
                     args.reps) if sums else float("nan")
        u, f = t_d + t_b, (t_ds + t_bs if sums else t_d + t_b)
        tot_u += 2 * u
        tot_f += 2 * f
        print(f"{name:18s} {nt:5d} {t_d:8.1f} {t_ds:8.1f} {t_b:8.1f} {t_bs:8.1f} {u:8.1f} {f:8.1f}", flush=True)
    print(f"per step (x2 domains, one block per stage shown): unfused {tot_u:.0f} us, fused {tot_f:.0f} us")


if __name__ == "__main__":
    main()
