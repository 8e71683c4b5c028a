#!/usr/bin/env python3
"""Isolated timing of the BN passes at the c2 step's shapes (batch 4, layer1 129x257 /
layer2-4 65x129), through the library's own HBM timing ids (algorithmic bytes / event time).

    python tools/bn_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from adaptsegnet_amd import kernels as K  # noqa: E402

DEV = "cuda"
SHAPES = [  # (name, rows, C, mode) mode: "res" = bn3 (mask from y, dres), "x" = bn1/bn2 (mask from x)
    ("l1.bn3", 4 * 129 * 257, 256, "res"), ("l1.bn2", 4 * 129 * 257, 64, "x"),
    ("l3.bn3", 4 * 65 * 129, 1024, "res"), ("l3.bn2", 4 * 65 * 129, 256, "x"),
    ("l4.bn3", 4 * 65 * 129, 2048, "res"), ("l4.bn2", 4 * 65 * 129, 512, "x"),
]
REPS = 20


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    print(f"{'bn':8s} {'rows':>7s} {'C':>5s}  {'kernel':36s} {'us':>8s} {'GB/s':>7s}")
    for name, rows, c, mode in SHAPES:
        x = torch.randn(rows, c, device=DEV, generator=g)
        dy = torch.randn(rows, c, device=DEV, generator=g)
        w = torch.rand(c, device=DEV, generator=g) + 0.5
        b = torch.randn(c, device=DEV, generator=g) * 0.1
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        res = torch.randn(rows, c, device=DEV, generator=g) if mode == "res" else None
        y, mean, invstd = K.bn_fwd_train(x, w, b, rm, rv, 0.1, 1e-5, res=res, relu=True)
        dres = torch.empty_like(dy) if mode == "res" else None
        for _ in range(3):
            K.bn_bwd(dy, y if mode == "res" else None, x, w, mean, invstd, relu=True, dres=dres, bias=b)
        torch.cuda.synchronize()
        K.timing_enable(-1)
        K.timing_enable(-1, enable=False)   # resets the record
        K.timing_enable_mem(True)
        for _ in range(REPS):
            K.bn_fwd_train(x, w, b, rm, rv, 0.1, 1e-5, res=res, relu=True, out=y)
            K.bn_bwd(dy, y if mode == "res" else None, x, w, mean, invstd, relu=True, dres=dres, bias=b)
        torch.cuda.synchronize()
        K.timing_enable_mem(False)
        for kid, kname in K.MEM_KERNELS.items():
            ms, by, n = K.timing_read_id(kid)
            if n:
                print(f"{name:8s} {rows:7d} {c:5d}  {kname:36s} {ms / n * 1e3:8.1f} {by / (ms / 1e3) / 1e9:7.0f}")


if __name__ == "__main__":
    main()
