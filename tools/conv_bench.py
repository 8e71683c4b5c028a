#!/usr/bin/env python3
"""Per-shape timing of every distinct conv product in one c2 adversarial step.

    python tools/conv_bench.py [--batch 4] [--reps 5]

Prints, for each (conv geometry, op) of DeeplabMulti + FCDiscriminator at 1024x512, the
kernel selector, K-split, launches per step, average time and TFLOP/s, then the step total.
Used to iterate on the igemm kernels without running the whole step.
"""
from __future__ import annotations

import argparse
import collections
import dataclasses
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from adaptsegnet_amd import engine  # noqa: E402
from adaptsegnet_amd import kernels as K  # noqa: E402


def _terms(t):
    """The pixel-interleaved F32X3 term images [..., 3, C] of an fp32 NHWC tensor (bn.hip x3_off)."""
    hi = t.to(torch.bfloat16)
    r = t - hi.float()
    mid = r.to(torch.bfloat16)
    return torch.stack([hi, mid, (r - mid.float()).to(torch.bfloat16)], dim=-2).contiguous()


def shapes(batch, W=1024, H=512):
    """(conv geometry, op set) -> [count, name] for one domain's G pass and D passes."""
    """(name, geom, n, h, w, ops, count/step, input strides or None)."""
    out = collections.OrderedDict()

    def add(name, g, n, h, w, ops, count, st=None):
        # thin input convs run channel-padded (engine._wgrad_padded / _FCDiscriminatorFn):
        # timed as the engine runs them (pad copies included), FLOPs of the unpadded geometry
        key = (g, n, h, w, ops, st)
        if key in out:
            out[key][0] += count
        else:
            out[key] = [count, name]

    # generator, 2 passes (source + target), single-level: layer5 fwd only
    h, w = H, W
    add("stem", K.ConvGeom(3, 64, 7, 7, 2, (3,), (1,)), batch, h, w, (0, 2), 2, (3 * h * w, h * w, w, 1))
    h, w = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1       # stem 7x7/2 p3
    h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1       # maxpool 3x3/2 p1
    cin = 64
    for li, (planes, nblk, stride, dil) in enumerate(((64, 3, 1, 1), (128, 4, 2, 1), (256, 23, 1, 2), (512, 3, 1, 4)), 1):
        if li == 4:
            add("aspp5", K.ConvGeom(1024, 19, 3, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24)), batch, h, w, (0,), 2)
        for b in range(nblk):
            s = stride if b == 0 else 1
            bin_ = cin if b == 0 else planes * 4
            g1 = K.ConvGeom(bin_, planes, 1, 1, s)
            add(f"l{li}.conv1", g1, batch, h, w, (0, 1, 2), 2)
            oh, ow = g1.out_hw(h, w)
            add(f"l{li}.conv2", K.ConvGeom(planes, planes, 3, 3, 1, (dil,), (dil,)), batch, oh, ow, (0, 1, 2), 2)
            add(f"l{li}.conv3", K.ConvGeom(planes, planes * 4, 1, 1), batch, oh, ow, (0, 1, 2), 2)
            if b == 0:
                add(f"l{li}.ds", K.ConvGeom(bin_, planes * 4, 1, 1, s), batch, h, w, (0, 1, 2), 2)
            h, w = oh, ow
        cin = planes * 4
    add("aspp6", K.ConvGeom(2048, 19, 3, 3, 1, (6, 12, 18, 24), (6, 12, 18, 24)), batch, h, w, (0, 1, 2), 2)
    # discriminator: fwd x3, dgrad x(1 + 2 for convs 2..5), wgrad x2
    h, w = H, W
    chans = (19, 64, 128, 256, 512, 1)
    for i in range(5):
        g = K.ConvGeom(chans[i], chans[i + 1], 4, 4, 2, (1,), (1,))
        st = (19 * h * w, 1, w * 19, 19) if i == 0 else None
        add(f"D.conv{i + 1}", g, batch, h, w, (0,), 3, st)
        add(f"D.conv{i + 1}", g, batch, h, w, (1,), 1 if i == 0 else 3)
        add(f"D.conv{i + 1}", g, batch, h, w, (2,), 2, st)
        h, w = g.out_hw(h, w)
    return out


def vgg_shapes(batch, W=1024, H=512):
    """config c4: DeeplabVGG (model/deeplab_vgg.py) per-shape products of one step (2 domains:
    2 forwards, 2 data gradients, 2 weight gradients; conv1_1 has no data gradient), then the
    discriminator's as in ``shapes``."""
    from adaptsegnet_amd.model import deeplab_vgg as V
    out = collections.OrderedDict()
    h, w = H, W
    specs = list(V._VGG_FEATURES) + [("C", 512, 1024, 4), ("R",), ("C", 1024, 1024, 4), ("R",)]
    i = 0
    for spec in specs:
        if spec[0] == "C":
            _, ci, co, d = spec
            g = K.ConvGeom(ci, co, 3, 3, 1, (d,), (d,))
            st = (3 * h * w, h * w, w, 1) if ci == 3 else None
            ops = (0, 2) if ci == 3 else (0, 1, 2)
            key = (g, batch, h, w, ops, st)
            if key in out:
                out[key][0] += 2
            else:
                out[key] = [2, f"vgg.c{i}"]
            i += 1
        elif spec[0] == "P":
            h, w = h // 2, w // 2
    out[(K.ConvGeom(1024, 19, 3, 3, 1, (6, 12), (6, 12)), batch, h, w, (0, 1, 2), None)] = [2, "vgg.aspp"]
    for k, v in shapes(batch, W, H).items():
        if v[1].startswith("D."):
            out[k] = v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--filter", default="")
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--math", choices=("f32", "f32x3", "f32x3_presplit", "bf16"), default="f32")
    ap.add_argument("--model", choices=("multi", "vgg"), default="multi",
                    help="multi: DeeplabMulti (c2 shapes); vgg: DeeplabVGG (config c4, use --batch 8)")
    args = ap.parse_args()
    K.set_conv_math({"f32": K.MATH_F32, "f32x3": K.MATH_F32X3, "f32x3_presplit": K.MATH_F32X3_PRESPLIT,
                     "bf16": K.MATH_BF16}[args.math])
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    tot_ms, tot_fl = 0.0, 0.0
    per_op = collections.defaultdict(lambda: [0.0, 0.0])
    print(f"{'conv':<10} {'op':>3} {'n':>2} {'hxw':>9} {'cin':>5} {'cout':>5} {'k':>2} {'sel':>4} {'spl':>3} "
          f"{'cnt':>4} {'avg us':>9} {'TF/s':>7} {'kern us':>9} {'kTF/s':>7}")
    table = (vgg_shapes if args.model == "vgg" else shapes)(args.batch, args.width, args.height)
    for (g, n, h, w, ops, st), (count, name) in table.items():
        if args.filter and args.filter not in name:
            continue
        oh, ow = g.out_hw(h, w)
        if st is None:
            x = torch.randn(n, h, w, g.cin, device=dev)
        else:
            x = torch.randn(n, g.cin, h, w, device=dev).permute(0, 2, 3, 1).contiguous() \
                if st[1] == 1 else torch.randn(n, g.cin, h, w, device=dev)
        ws = [torch.randn(g.cout, g.kh, g.kw, g.cin, device=dev) * 0.01 for _ in range(g.nseg)]
        # only the ASPP classifiers and the discriminator convs carry a bias
        has_bias = name.startswith(("aspp", "D.", "vgg."))
        bs = [torch.randn(g.cout, device=dev) for _ in range(g.nseg)] if has_bias else None
        dy = torch.randn(n, oh, ow, g.cout, device=dev)
        dws = [torch.zeros_like(t) for t in ws]
        dbs = [torch.zeros_like(t) for t in bs] if has_bias else None
        pad_wgrad = g.cin % 4 != 0                     # D.conv1 (Cin 20), stem (Cin 4)
        xn = x.permute(0, 3, 1, 2) if x.dim() == 4 and x.shape[-1] == g.cin else x
        # the products the engine runs on term images under F32X3 (engine.x3_forward_terms /
        # X3_BWD_TERMS: the layer 3-4 conv2 forward, data and weight gradients), timed so
        tf = st is None and name.endswith("conv2") and engine.x3_forward_terms(g)
        tb = tf and engine.X3_BWD_TERMS >= 2
        tw = (tf and engine.X3_BWD_TERMS >= 1) or (st is None and name.endswith("conv2") and
                                                    engine.x3_wgrad_terms(g))
        xt = _terms(x) if tf or tw else None
        dyt = _terms(dy) if tb or tw else None
        for op in ops:
            def run():
                if op == 0 and tf:
                    K.conv_fwd(g, None, n, h, w, ws, bs, xb=xt)
                elif op == 0:
                    K.conv_fwd(g, x, n, h, w, ws, bs, strides=st)
                elif op == 1 and tb:
                    K.conv_dgrad(g, None, n, h, w, ws, dyb=dyt)
                elif op == 1:
                    K.conv_dgrad(g, dy, n, h, w, ws)
                elif op == 2 and tw:
                    K.conv_wgrad(g, None, None, n, h, w, dws, dbs, dyb=dyt, xb=xt)
                elif pad_wgrad:
                    c4 = (g.cin + 3) // 4 * 4
                    xp = K.to_nhwc_pad(xn, c4)
                    dwp = K.zero_(torch.empty(g.cout, g.kh, g.kw, c4, device=dev))
                    K.conv_wgrad(dataclasses.replace(g, cin=c4), dy, xp, n, h, w, [dwp], dbs,
                                 strides=K.nhwc_strides(n, h, w, c4))
                    K.to_nhwc_pad(dwp.permute(0, 3, 1, 2)[:, :g.cin], g.cin, out=dws[0], accumulate=True)
                else:
                    K.conv_wgrad(g, dy, x, n, h, w, dws, dbs, strides=st)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            # the GEMM kernel alone (the library's own hipEvent bracket: no weight pack,
            # activation copy or split-K reduce)
            K.timing_enable(-1, True)
            for _ in range(args.reps):
                run()
            torch.cuda.synchronize()
            kms, _, kn = K.timing_read()
            K.timing_enable(-1, False)
            kus = 1e3 * kms / max(1, args.reps)
            fl = g.flops(n, h, w)
            if op == 2 and pad_wgrad:
                c4 = (g.cin + 3) // 4 * 4
                sel, sp = K.conv_kernel_id(dataclasses.replace(g, cin=c4), n, h, w, op, K.nhwc_strides(n, h, w, c4))
            else:
                sel, sp = K.conv_kernel_id(g, n, h, w, op, st, copies=(tf, tb, tw)[op])
            c = count[op] if isinstance(count, dict) else count
            tot_ms += ms * c
            tot_fl += fl * c
            per_op[op][0] += ms * c
            per_op[op][1] += fl * c
            print(f"{name:<10} {op:>3} {n:>2} {h:>4}x{w:<4} {g.cin:>5} {g.cout:>5} {g.kh:>2} {sel:>4} {sp:>3} "
                  f"{c:>4} {ms * 1e3:9.1f} {fl / ms / 1e9:7.1f} {kus:9.1f} {fl / max(kus, 1e-3) / 1e6:7.1f}", flush=True)
    for op, (ms, fl) in sorted(per_op.items()):
        print(f"op {op}: {ms:8.2f} ms/step  {fl / 1e12:6.3f} TFLOP  {fl / ms / 1e9:6.1f} TF/s")
    print(f"TOTAL conv: {tot_ms:8.2f} ms/step, {tot_fl / 1e12:.3f} TFLOP, {tot_fl / tot_ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
