#!/usr/bin/env python3
"""Isolated timing of the BN passes at the c2 step's shapes (batch 4, layer1 129x257 /
layer2-4 65x129), through the library's own HBM timing ids (algorithmic bytes / event time).

    python tools/bn_bench.py [--bf16]

--bf16: the c5 program's storage (bf16 activations x / residual / y, fp32 gradients in, the
backward writing only the bf16 copy of dx and the fp32 residual gradient).
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
    lp = "--bf16" in sys.argv
    if lp:
        K.set_conv_math(K.MATH_BF16)   # bf16 activation storage is the bf16 maths' (c5)
    g = torch.Generator(device=DEV).manual_seed(0)
    print(f"{'bn':8s} {'rows':>7s} {'C':>5s}  {'kernel':36s} {'us':>8s} {'GB/s':>7s}")
    for name, rows, c, mode in SHAPES:
        x = torch.randn(rows, c, device=DEV, generator=g)
        dy = torch.randn(rows, c, device=DEV, generator=g)
        w = torch.rand(c, device=DEV, generator=g) + 0.5
        b = torch.randn(c, device=DEV, generator=g) * 0.1
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        res = torch.randn(rows, c, device=DEV, generator=g) if mode == "res" else None
        if lp:
            x = x.to(torch.bfloat16)
            res = res.to(torch.bfloat16) if res is not None else None
        dres = torch.empty_like(dy) if mode == "res" else None

        def fwd():
            if lp:
                return K.bn_fwd_train(x, w, b, rm, rv, 0.1, 1e-5, res=res, relu=True, bf16_out=True,
                                      fp32_out=False)[3]
            return K.bn_fwd_train(x, w, b, rm, rv, 0.1, 1e-5, res=res, relu=True, out=y)[0]

        def bwd():
            K.bn_bwd(dy, y if mode == "res" else None, x, w, mean, invstd, relu=True, dres=dres, bias=b,
                     bf16_out=lp, fp32_out=not lp)

        if lp:
            _, mean, invstd, y = K.bn_fwd_train(x, w, b, rm, rv, 0.1, 1e-5, res=res, relu=True, bf16_out=True,
                                                fp32_out=False)
        else:
            y, mean, invstd = K.bn_fwd_train(x, w, b, rm, rv, 0.1, 1e-5, res=res, relu=True)
        for _ in range(3):
            bwd()
        torch.cuda.synchronize()
        K.timing_enable(-1)
        K.timing_enable(-1, enable=False)   # resets the record
        K.timing_enable_mem(True)
        for _ in range(REPS):
            fwd()
            bwd()
        torch.cuda.synchronize()
        K.timing_enable_mem(False)
        for kid, kname in K.MEM_KERNELS.items():
            ms, by, n = K.timing_read_id(kid)
            if n:
                print(f"{name:8s} {rows:7d} {c:5d}  {kname:36s} {ms / n * 1e3:8.1f} {by / (ms / 1e3) / 1e9:7.0f}")


if __name__ == "__main__":
    main()
