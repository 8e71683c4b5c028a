#!/usr/bin/env python3
"""Benchmark: AdaptSegNet adversarial-train images/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

One "step" = one full adversarial iteration of train_gta2cityscapes_multi.py on the HIP
engine (2 G forwards, 2 G backwards, D forwards/backwards, SGD + Adam) over one synthetic
batch already resident in HBM.  Default workload = BASELINE config c2: single-level,
batch 4 per GPU, source and target 1024x512, Vanilla GAN, fp32 (the reference's dtype).
``value`` = (source, target) pairs per second over all ranks (weak scaling: batch per GPU
is fixed).  Rank 0 prints ONE JSON line.

Conv math: the fp32 configs run F32X3 by default (fp32-accurate convs on the bf16 MFMA through
exact three-term bf16 operand splits, six bf16 products per fp32 product; conv_x3.hpp),
``--conv-math f32`` the fp32-input MFMA kernels; c5 runs bf16 operands.

roofline: the dominant implicit-GEMM conv kernel symbol (the most kernel execution time per
step, from execution-time events of every conv launch of one untimed step) is launched with
hipExtLaunchKernel start/stop events inside the library during the timed steps, which time the
kernel's own execution as rocprofv3 does; achieved = its
algorithmic FLOPs / its summed execution time, against that kernel's MFMA ceiling: the fp32 MFMA
peak (157.3 TFLOP/s) for the fp32-input kernels, the bf16 dense peak / 6 (419.4 TFLOP/s of
fp32 products) for F32X3, the bf16 dense peak (2516.6) for bf16.
cpu_baseline: the oracle (stock-PyTorch CPU restatement of the reference step, the
reference's own arithmetic) timed on this host for ONE single-level step at batch 1.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X: 256 CU x 2.4 GHz x 256 FLOP/clk/CU (MI355X_MICROARCH.md)
METRIC = "adversarial-train images/sec at 1024×512, DeeplabMulti+D, 1/2/4/8 MI355X"

HBM_PEAK_GBS = 8000.0           # MI355X HBM3E (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # 256 CU x 2.4 GHz x 4096 FLOP/clk/CU (v_mfma_f32_32x32x16_bf16), dense

CONFIGS = {
    # name: (level, gan, batch/GPU, source (W,H), target (W,H), generator, conv math)
    "c2": ("single-level", "Vanilla", 4, (1024, 512), (1024, 512), "DeeplabMulti", "f32"),
    "c3": ("multi-level", "Vanilla", 2, (1280, 720), (1024, 512), "DeeplabMulti", "f32"),
    "c4": ("single-level", "Vanilla", 8, (1024, 512), (1024, 512), "DeeplabVGG", "f32"),
    # BASELINE c5: multi-level LS-GAN, bf16 conv math (autocast semantics), batch/GPU 4
    "c5": ("multi-level", "LS", 4, (1280, 720), (1024, 512), "DeeplabMulti", "bf16"),
}


def conv_inventory(model, D, level, batch, src_wh, tgt_wh, tsize, products=None, nbytes=None, d_reuse=True,
                   first_head=False):
    """Algorithmic conv FLOPs of one step, keyed by igemm kernel selector.  ``products``
    (a set), when given, also collects every (op, selector, split-K?) the step launches
    (host-side planning only: tests/test_conv_coverage.py runs it without a GPU).  ``nbytes``
    (a dict), when given, receives each selector's algorithmic HBM bytes per step: every
    operand read once and the output written once, fp32 (4 B; bf16 math 2 B) per element.
    ``d_reuse``: StepConfig.d_reuse — D's own step on the target reuses the adversarial forward.
    ``first_head``: single-level with the discarded layer5 head computed (second_head_only off)."""
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd import engine
    inv = {}

    copies = engine.bf16_operands()   # the Bottleneck products get their operand copies

    def add(geom, n, h, w, op, strides=None, count=1, algo=None, cp=False, terms=False):
        # geom: the geometry the engine launches; algo: the reference's (unpadded) one, whose
        # FLOPs are counted; cp: the engine passes the operand copies (engine.block_forward /
        # block_backward under bf16_operands); terms: it passes them for this product alone
        # (engine.x3_forward_terms)
        kid, sp = K.conv_kernel_id(geom, n, h, w, op, strides, copies=(cp and copies) or terms)
        inv[kid] = inv.get(kid, 0.0) + count * (algo or geom).flops(n, h, w)
        if nbytes is not None:
            g = algo or geom
            oh, ow = g.out_hw(h, w)
            eb = 2 if K.get_conv_math() == K.MATH_BF16 else 4
            elems = n * h * w * g.cin + g.cout * g.cin * g.kh * g.kw * len(g.pads) + n * oh * ow * g.cout
            nbytes[kid] = nbytes.get(kid, 0.0) + count * eb * elems
        if products is not None:
            products.add((op, kid, sp > 1))

    def vgg_pass(wh):
        w, h = wh
        st = (3 * h * w, h * w, w, 1)
        # the term images engine._DeeplabVGGFn makes (engine.VGG_TERMS / VGG_TERMS_MIN_C): conv i's
        # input terms when its Cin qualifies, its output-gradient terms when its Cout does (the
        # last conv's always, from the classifier's data gradient)
        vt, thr = engine.vgg_terms(), engine.VGG_TERMS_MIN_C
        prog = model.conv_program()
        for i, (conv, pool) in enumerate(prog):
            g = conv.geom()
            xt = vt > 0 and i > 0 and g.cin % 8 == 0 and g.cin >= thr
            dt = vt > 0 and (i == len(prog) - 1 or (i > 0 and g.cout % 8 == 0 and g.cout >= thr))
            add(g, batch, h, w, 0, st, terms=vt >= 2 and xt)
            if i > 0:
                add(g, batch, h, w, 1, terms=vt >= 2 and dt)
            if g.cin % 4:   # conv1_1: weight gradient on the 4-channel padded input
                add(dataclasses.replace(g, cin=4), batch, h, w, 2, (4 * h * w, 1, 4 * w, 4), algo=g)
            else:
                add(g, batch, h, w, 2, st, terms=xt and dt)
            h, w = g.out_hw(h, w)
            if pool:
                h, w = h // 2, w // 2
            st = None
        gc = engine._branches_geom(model.classifier_branches())
        for op in (0, 1, 2):
            add(gc, batch, h, w, op)

    def g_pass(wh, backward, heads_bwd):
        if getattr(model, "single_output", False):
            return vgg_pass(wh)
        w, h = wh
        gs = model.conv1.geom()
        add(gs, batch, h, w, 0, (3 * h * w, h * w, w, 1))
        if backward:   # weight gradient on the 4-channel padded input (engine._wgrad_padded)
            add(dataclasses.replace(gs, cin=4), batch, h, w, 2, (4 * h * w, 1, 4 * w, 4), algo=gs)
        h, w = gs.out_hw(h, w)
        h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
        for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4), 1):
            if li == 4 and ("l5" in heads_bwd or first_head):   # (single-level: layer5 not computed)
                g5 = engine.aspp_geom(model.layer5)
                add(g5, batch, h, w, 0)
                if backward and "l5" in heads_bwd:
                    add(g5, batch, h, w, 1)
                    add(g5, batch, h, w, 2)
            for bi, blk in enumerate(layer):
                first = li == 1 and bi == 0   # its input (the max-pool output) has no copy
                convs = [(blk.conv1, h, w, not first)]
                oh, ow = blk.conv1.geom().out_hw(h, w)
                convs += [(blk.conv2, oh, ow, True), (blk.conv3, oh, ow, True)]
                if blk.downsample is not None:
                    convs.append((blk.downsample[0], h, w, not first))
                for conv, ch, cw, xcp in convs:
                    fwd_terms = conv is blk.conv2 and not copies and engine.x3_forward_terms(conv.geom())
                    add(conv.geom(), batch, ch, cw, 0, cp=xcp, terms=fwd_terms)
                    if backward and (li < 4 or "l6" in heads_bwd):
                        # engine.block_backward: conv2's backward on term images (X3_BWD_TERMS)
                        c3t = (conv is blk.conv3 and not copies and engine.X3_BWD_TERMS >= 3 and
                               engine.x3_forward_terms(blk.conv2.geom()) and conv.geom().cin % 32 == 0)
                        add(conv.geom(), batch, ch, cw, 1, cp=True,
                            terms=(fwd_terms and engine.X3_BWD_TERMS >= 2) or c3t)
                        wt2 = conv is blk.conv2 and not copies and engine.x3_wgrad_terms(conv.geom())
                        add(conv.geom(), batch, ch, cw, 2, cp=xcp,
                            terms=(fwd_terms and engine.X3_BWD_TERMS >= 1) or c3t or wt2)
                h, w = oh, ow
        g6 = engine.aspp_geom(model.layer6)
        add(g6, batch, h, w, 0)
        if backward and "l6" in heads_bwd:
            add(g6, batch, h, w, 1)
            add(g6, batch, h, w, 2)

    def d_pass(wh, dgrad_input, wgrad, forward=True):
        w, h = wh
        for i, conv in enumerate(D._convs()):
            g = conv.geom()
            if i == 0:   # Cin 19; weight gradient on a 20-channel padded copy (engine._wgrad_padded)
                if forward:
                    add(g, batch, h, w, 0, (19 * h * w, 1, w * 19, 19))
                if dgrad_input:
                    add(g, batch, h, w, 1)
                if wgrad:
                    add(dataclasses.replace(g, cin=20), batch, h, w, 2, (20 * h * w, 1, w * 20, 20), algo=g)
            else:
                if forward:
                    add(g, batch, h, w, 0)
                add(g, batch, h, w, 1)
                if wgrad:
                    add(g, batch, h, w, 2)
            h, w = g.out_hw(h, w)

    heads = {"l6"} if level == "single-level" else {"l5", "l6"}
    nD = 1 if level == "single-level" else 2
    g_pass(src_wh, True, heads)
    g_pass(tgt_wh, True, heads)
    for _ in range(nD):
        d_pass(tsize, True, False)        # G step through the frozen D
        d_pass(src_wh, False, True)       # D step, source
        d_pass(tsize, False, True, not d_reuse)   # D step, target (d_reuse: the G step's forward)
    return inv


# kernel selector (adaptseg_conv2d_kernel_id) -> the kernel template rocprofv3 reports
_CFG = {0: (128, 128, 2, 2, 32), 1: (256, 32, 4, 1, 32), 2: (32, 256, 1, 4, 32), 3: (64, 256, 1, 4, 32),
        4: (256, 64, 4, 1, 16), 5: (64, 64, 2, 2, 32), 6: (128, 128, 2, 2, 16), 7: (256, 128, 4, 2, 32),
        8: (128, 128, 2, 2, 16)}


def kernel_peak(sel):
    """(MFMA ceiling in TFLOP/s of algorithmic products, family) of a kernel selector."""
    if sel % 100 in (86, 87, 88, 89, 95, 96):
        return BF16_MFMA_PEAK_TFLOPS / 6, "f32x3 (6 bf16 MFMA products per fp32 product)"
    if sel % 100 >= 90 or sel % 100 == 85:
        return BF16_MFMA_PEAK_TFLOPS, "bf16"
    return FP32_MFMA_PEAK_TFLOPS, "fp32-input MFMA"


def selector_symbol(sel):
    op, cfg, var = sel // 100, sel // 10 % 10, sel % 10
    if sel % 100 in (95, 96):
        return f"igemm_x3_kernel<{op}, {'true' if var == 6 else 'false'}>"
    if sel % 100 == 85:   # bf16 LDS-DMA 256x256x64, two stages
        if op == 2:
            return "igemm_bf16g_wgrad_kernel<256, 256, 2>"
        return f"igemm_bf16g_kernel<{op}, 256, 256, 64, false, 2>"
    if sel % 100 in (86, 87):   # F32X3, the same tiles with the fp32 operands split in-kernel
        if op == 2:
            return f"igemm_x3hw_kernel<{256 if var == 6 else 128}>"
        return f"igemm_x3h_kernel<{op}, {'true' if var == 7 else 'false'}>"
    if sel % 100 in (88, 89):   # F32X3, 256x128x32 tiles on pre-split images (conv_x3r.hpp)
        if op == 2:
            return f"igemm_x3r_wgrad_kernel<{256 if var == 8 else 128}>"
        return f"igemm_x3r_kernel<{op}, {'true' if var == 9 else 'false'}>"
    if sel % 100 in (92, 93) and op == 1:   # bf16 LDS-DMA stride-2 data gradient (parity classes)
        bm, bn = (128, 256) if var == 2 else (256, 128)
        return f"igemm_bf16g_kernel<1, {bm}, {bn}, 32, true>"
    if sel % 100 in (94, 97, 98, 99):   # the bf16 LDS-DMA kernels (conv_bf16g.hpp)
        if op == 2:
            return f"igemm_bf16g_wgrad_kernel<{256 if var == 8 else 128}>"
        bm, bn = (128, 256) if var in (4, 7) else (256, 128)
        return f"igemm_bf16g_kernel<{op}, {bm}, {bn}, {64 if var in (7, 8) else 32}>"
    if cfg == 9:
        return f"igemm_bf16_kernel<{op}, {'true' if var & 1 else 'false'}, {256 if var & 2 else 128}>"
    bm, bn, wm, wn, bk = _CFG[cfg]
    b = lambda v: "true" if v else "false"  # noqa: E731
    if var >= 4:
        v = var - 4
        minb = 3 if cfg == 8 else 1   # __launch_bounds__ min-blocks template argument
        return (f"igemm_fast_kernel<{op}, {bm}, {bn}, {wm}, {wn}, {bk}, {b(v & 4)}, {b(v & 2)}, "
                f"{b(v & 1)}, {minb}>")
    return f"igemm_kernel<{op}, {bm}, {bn}, {wm}, {wn}, {b(var & 2)}, {b(var & 1)}>"


def pmc_traffic(config, sel):
    """Per-launch HBM-side bytes of the dominant kernel from the committed PMC passes
    (tools/gpu_traffic.sh + tools/traffic_summary.py over this same bench command):
    profiles/rN/pmc/traffic_<config>[_<kernel>].json, newest round first."""
    import glob
    for rnd in ("r6", "r5", "r4", "r3", "r2", "r1"):
        for path in sorted(glob.glob(os.path.join(REPO, "profiles", rnd, "pmc", f"traffic_{config}*.json"))):
            try:
                d = json.load(open(path))
            except (OSError, ValueError):
                continue
            if d.get("kernel") == selector_symbol(sel) and d.get("traffic_bytes_per_launch"):
                return float(d["traffic_bytes_per_launch"]), os.path.relpath(path, REPO)
    return None, None


def cpu_baseline(threads):
    """The oracle's step on `threads` host cores, fp32, batch 1 (SURVEY §8(d) CPU reference):

    * c2 shape (single-level Vanilla, 1024x512 source and target): 1 warm-up + 2 timed steps,
      `value` = images/s of the timed steps;
    * c3 shape (multi-level Vanilla, source 1280x720, target 1024x512, D1 + D2): 1 warm-up +
      2 timed steps, reported as `c3_step_s`;
    * BASELINE config c1 (forward + CrossEntropy2d, 1x3x321x321): 1 warm-up + 1 timed.
    The warm-up keeps oneDNN primitive creation out of the timed steps.
    """
    from oracle import reference_torch as R
    torch.set_num_threads(threads)

    def run(level, src, tgt, n_timed):
        G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=torch.float32, trainable=R.g_trainable)
        d = lambda seed: R.to_torch(R.det_state(R.d_specs(), seed), dtype=torch.float32,
                                    trainable=lambda k: True)
        D1 = d(2001) if level == "multi-level" else None
        D2 = d(2002)
        cfg = dict(level=level, gan="Vanilla", input_size=src, input_size_target=tgt)
        opts = R.make_optimizers(G, D1, D2, R.DEFAULT_CFG | cfg)
        xs = torch.from_numpy(R.det_images((1, 3, src[1], src[0]), 1)).float()
        lab = torch.from_numpy(R.det_labels((1, src[1], src[0]), 2))
        xt = torch.from_numpy(R.det_images((1, 3, tgt[1], tgt[0]), 3)).float()
        R.oracle_step(G, D1, D2, opts, cfg, 0, [(xs, lab, xt)])          # warm-up
        t0 = time.perf_counter()
        for it in range(n_timed):
            R.oracle_step(G, D1, D2, opts, cfg, 1 + it, [(xs, lab, xt)])
        return (time.perf_counter() - t0) / n_timed, G

    c2_s, G = run("single-level", (1024, 512), (1024, 512), 2)
    c3_s, _ = run("multi-level", (1280, 720), (1024, 512), 2)
    x1 = torch.from_numpy(R.det_images((1, 3, 321, 321), 5)).float()
    l1 = torch.from_numpy(R.det_labels((1, 321, 321), 6))
    times = []
    with torch.no_grad():
        for _ in range(2):
            t1 = time.perf_counter()
            R.cross_entropy2d(R.g_forward(G, x1, (321, 321), train=True)[1], l1)
            times.append(time.perf_counter() - t1)
    return {"value": 1.0 / c2_s, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": "oracle/reference_torch.py step (stock PyTorch CPU fp32), batch 1: c2 shape "
                      f"single-level 1024x512, 1 warm-up + 2 timed, {c2_s:.2f} s/step",
            "c3_step_s": c3_s,
            "c3_sample": "multi-level Vanilla, source 1280x720 + target 1024x512, batch 1, "
                         "1 warm-up + 2 timed",
            "c3_images_per_s": 1.0 / c3_s,
            "c1_forward_ce_s": times[-1],
            "calibration": "the port times within +3.3 % (step) / -3.2 % (c1) of the reference's own "
                           "modules on the same 8 cores, interleaved best of 6 "
                           "(profiles/r4/cpu_calibration.json)"}


def init_distributed(backend, local, init=None, set_device=None):
    """One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_*): bind the local GPU and create the process group.  ``nccl`` (= RCCL over xGMI)
    runs its collectives on a HIGH-priority stream, like the step's main chain
    (StepConfig.main_priority): the generator's bucketed all-reduces, launched from inside its
    backward, must not queue behind the weight-gradient / discriminator kernels.  ``gloo`` only
    rehearses the multi-rank path on one GPU.  ``init`` / ``set_device`` default to
    torch.distributed.init_process_group / torch.cuda.set_device (tests pass stubs)."""
    init = init or dist.init_process_group
    (set_device or torch.cuda.set_device)(local)
    if backend == "nccl":
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        init("nccl", device_id=torch.device("cuda", local), pg_options=opts)
    else:
        init("gloo")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="c2 (default, BASELINE metric at N=1), c3 multi-level, c4 DeeplabVGG, "
                         "c5 multi-level LS bf16 batch 4")
    ap.add_argument("--batch", type=int, default=None, help="override batch per GPU")
    ap.add_argument("--conv-math", default="f32x3", choices=("f32x3", "f32x3_presplit", "f32"),
                    help="conv arithmetic of the fp32 configs: f32x3 (default, fp32-accurate on the "
                         "bf16 MFMA) or f32 (the fp32-input MFMA kernels)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--overlap", default="auto", choices=("auto", "on", "off"),
                    help="run the target-domain pass on a second stream, overlapping the source "
                         "backward (StepConfig.overlap_domains; auto: on for DeeplabMulti)")
    ap.add_argument("--overlap-d", action="store_true",
                    help="run the discriminator step on its own stream beside the last generator "
                         "backward (StepConfig.overlap_d)")
    ap.add_argument("--no-d-reuse", action="store_true",
                    help="run D again on the target prediction for its own step instead of reusing "
                         "the adversarial forward (StepConfig.d_reuse off)")
    ap.add_argument("--both-heads", action="store_true",
                    help="single-level: compute the discarded first head too (StepConfig.second_head_only off)")
    ap.add_argument("--target-first", action="store_true",
                    help="with the domain overlap, enqueue the target forward before the source "
                         "backward (StepConfig.target_first)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the multi-rank path with several ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        init_distributed(args.backend, local)
    dev = torch.device("cuda", local)

    from adaptsegnet_amd import engine
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, DeeplabVGG, FCDiscriminator
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig

    level, gan, batch, src_wh, tgt_wh, gen, math = CONFIGS[args.config]
    conv_math = "bf16" if math == "bf16" else args.conv_math
    K.set_conv_math({"bf16": K.MATH_BF16, "f32x3": K.MATH_F32X3, "f32x3_presplit": K.MATH_F32X3_PRESPLIT,
                     "f32": K.MATH_F32}[conv_math])
    if args.batch:
        batch = args.batch
    torch.manual_seed(1338 + rank)
    model = (DeeplabMulti if gen == "DeeplabMulti" else DeeplabVGG)(num_classes=19).to(dev)
    D1 = FCDiscriminator(num_classes=19).to(dev) if level == "multi-level" else None
    D2 = FCDiscriminator(num_classes=19).to(dev)
    if world > 1:  # identical initial weights on every rank (DDP's initial broadcast)
        for m in (model, D1, D2):
            if m is not None:
                for t in list(m.parameters()) + list(m.buffers()):
                    dist.broadcast(t.data, 0)
    model.train()
    scfg = StepConfig(level=level, gan=gan, input_size=src_wh, input_size_target=tgt_wh,
                      overlap_domains={"auto": "auto", "on": True, "off": False}[args.overlap],
                      overlap_d=args.overlap_d, target_first=args.target_first,
                      d_reuse=not args.no_d_reuse, second_head_only=not args.both_heads)
    trainer = AdaptSegTrainer(model, D1, D2, scfg)
    tsize = trainer._target_size()

    g = torch.Generator().manual_seed(1338 + rank)
    xs = (torch.rand(batch, 3, src_wh[1], src_wh[0], generator=g) * 273.7 - 122.7).to(dev)
    lab = torch.randint(0, 19, (batch, src_wh[1], src_wh[0]), generator=g)
    lab[torch.rand(lab.shape, generator=g) < 0.1] = 255
    lab = lab.to(dev)
    xt = (torch.rand(batch, 3, tgt_wh[1], tgt_wh[0], generator=g) * 273.7 - 122.7).to(dev)
    batches = [(xs, lab, xt)]

    for i in range(args.warmup):
        trainer.step(i, batches)
    torch.cuda.synchronize()

    inv_bytes = {}
    inv = conv_inventory(model, D2, level, batch, src_wh, tgt_wh, tsize, nbytes=inv_bytes, d_reuse=scfg.d_reuse,
                         first_head=not scfg.second_head_only)
    step_flops = sum(inv.values())
    # the roofline kernel: the conv symbol with the most measured kernel time per step (below);
    # without the untimed timing step (--no-roofline) the one with the most algorithmic FLOPs
    dom = max(inv, key=inv.get)
    hbm = []
    if not args.no_roofline:
        # HBM-bound kernels (interp / loss / BN passes): hipEvent pairs around each of their
        # ~400 launches per step, over ONE extra untimed step — inside the timed region those
        # event pairs cost ~2 % of the step.  The timed region keeps only the dominant conv
        # kernel's events (the roofline below).
        # The same untimed step also brackets EVERY conv launch, for the per-kernel rooflines
        # of the largest symbols (roofline.by_kernel); the timed region records only `dom`.
        K.timing_enable(-1)
        K.timing_enable_mem(True)
        K.timing_enable_stream(True)
        trainer.step(args.warmup, batches)
        torch.cuda.synchronize()
        K.timing_enable_stream(False)
        K.timing_enable_mem(False)
        K.timing_enable(-1, enable=False)
        by_kernel = []
        # conv GEMMs: execution time (hipExtLaunchKernel events: the kernel's own start to end,
        # what rocprofv3 reports) ranks them; the stream time of the same launches (events
        # recorded around the launch in its stream: includes waiting for CU slots beside the
        # other streams' work) is reported beside it
        live = {sel: K.timing_read_id(sel) for sel in inv}
        live = {sel: t for sel, t in live.items() if t[2]}
        if live:
            dom = max(live, key=lambda sel: live[sel][0])
        for sel in sorted(live, key=lambda sel: live[sel][0], reverse=True)[:6]:
            ms_, _fl, n_ = live[sel]
            sms_, sn_ = K.timing_read_id_stream(sel)
            pk, fam = kernel_peak(sel)
            a_ = inv[sel] / (ms_ / 1e3) / 1e12   # algorithmic FLOPs of one step / summed launch time
            sa_ = inv[sel] / (sms_ / 1e3) / 1e12 if sms_ else None
            by_kernel.append({"kernel": selector_symbol(sel), "selector": sel, "achieved": a_, "peak": pk,
                              "unit": "TFLOP/s", "frac": a_ / pk, "kernel_family": fam,
                              "kernel_ms_per_step": ms_, "launches_per_step": n_, "avg_launch_ms": ms_ / n_,
                              "stream_ms_per_step": sms_, "stream_avg_launch_ms": sms_ / sn_ if sn_ else None,
                              "stream_frac": sa_ / pk if sa_ else None,
                              "algorithmic_tflop_per_step": inv[sel] / 1e12,
                              "flop_share_of_step": inv[sel] / step_flops})
        for kid, name in K.MEM_KERNELS.items():
            ms_, by_, n_ = K.timing_read_id(kid)
            if n_:
                gbs = by_ / (ms_ / 1e3) / 1e9
                hbm.append({"kernel": name, "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                            "algorithmic_bytes_per_launch": by_ / n_, "avg_launch_ms": ms_ / n_,
                            "launches_per_step": n_})
        # every event pair the timed steps record exists before them (one created inside the
        # timed region costs milliseconds: adaptseg_timing_reserve)
        K.timing_reserve(int(live.get(dom, (0, 0, 0))[2] * (args.steps + 1) * 1.25) + 64)
        K.timing_enable(dom)
    peak, family = kernel_peak(dom)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it0 = args.warmup + (0 if args.no_roofline else 1)   # after the HBM-timing step
    for i in range(args.steps):
        L = trainer.step(it0 + i, batches)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not args.no_roofline:
        K.timing_enable(dom, enable=False)
        k_ms, k_flops, k_launches = K.timing_read()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    losses = L.values()
    for k, v in losses.items():
        if not np.isfinite(v):
            raise RuntimeError(f"non-finite loss {k}={v}")

    ms_per_step = elapsed / args.steps * 1e3
    pairs = batch * world * args.steps
    out = {
        "metric": METRIC, "value": pairs / elapsed, "unit": "images/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": math,
        "data": "synthetic (U[-122.7,151] BGR-mean-subtracted pixels, uniform labels, 10% ignore=255)",
        "config": {"workload": f"{args.config}: {gen} {level} {gan}, batch/GPU {batch}, source "
                               f"{src_wh[0]}x{src_wh[1]}, target {tgt_wh[0]}x{tgt_wh[1]}",
                   "global_batch": batch * world, "parallelism": f"dp{world}",
                   "step_conv_tflop": step_flops / 1e12,
                   "step_conv_tflops_achieved": step_flops / (ms_per_step / 1e3) / 1e12,
                   "conv_math": conv_math,
                   "switches": engine.switches(),
                   "x3h_mode": K.get_x3h(), "g16_wide": K.get_g16_wide(),
                   "overlap_domains": trainer._overlap_domains(), "overlap_d": bool(scfg.overlap_d),
                   "target_first": bool(scfg.target_first), "d_reuse": bool(scfg.d_reuse),
                   "second_head_only": bool(scfg.second_head_only),
                   # algorithmic conv FLOPs / step time / (n_gpu x peak)
                   "step_conv_frac_of_peak": step_flops / (ms_per_step / 1e3) / 1e12 / peak,
                   # the same against a fixed denominator (the fp32 MFMA peak), comparable across
                   # conv maths and rounds (the line above divides by the dominant family's peak)
                   "step_conv_frac_of_fp32_peak": step_flops / (ms_per_step / 1e3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
                   "losses_last_step": losses,
                   # caching-allocator peak over the whole run (d_reuse keeps D's target-forward
                   # activations until D's own step: ADVICE r5; --no-d-reuse is the low-memory arm)
                   "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 1e9},
    }
    if not args.no_roofline and k_launches:
        avg_ms = k_ms / k_launches
        # algorithmic FLOPs from the step inventory (unpadded geometries): the library's own
        # count includes the zero channels of the channel-padded thin convs (D.conv1 runs
        # Cin 19 as 32), which are not the reference's work
        launched_flops = k_flops
        k_flops = inv[dom] * args.steps
        ach = k_flops / (k_ms / 1e3) / 1e12
        traffic, tsrc = pmc_traffic(args.config, dom)
        out["roofline"] = {"bound": "mfma", "achieved": ach, "peak": peak,
                           "unit": "TFLOP/s", "frac": ach / peak, "traffic": traffic,
                           "kernel_family": family,
                           "frac_of_fp32_mfma_peak": ach / FP32_MFMA_PEAK_TFLOPS,
                           "traffic_unit": "bytes/launch (L2 memory-side FETCH_SIZE x2 + WRITE_SIZE)",
                           "traffic_source": tsrc,
                           # operands read once + output written once, per launch: traffic well
                           # above it = operand re-reads (per tap / column tile, served by MALL)
                           "algorithmic_bytes_per_launch": inv_bytes.get(dom, 0.0) * args.steps / k_launches,
                           "traffic_over_algorithmic": (traffic / (inv_bytes[dom] * args.steps / k_launches)
                                                        if traffic and inv_bytes.get(dom) else None),
                           "algorithmic_flop_per_launch": k_flops / k_launches,
                           "launched_flop_per_launch": launched_flops / k_launches,
                           "kernel": selector_symbol(dom), "selector": dom,
                           "chosen_by": "most kernel execution time per step (by_kernel)",
                           "timing": "kernel execution (hipExtLaunchKernel start/stop events, as rocprofv3 "
                                     "reports kernel durations); by_kernel adds the stream time",
                           "launches_per_step": k_launches / args.steps,
                           "avg_launch_ms": avg_ms,
                           "flop_share_of_step": inv[dom] / step_flops,
                           # the six conv symbols with the most kernel time, live over the
                           # untimed step before the timed one
                           "by_kernel": by_kernel,
                           "by_kernel_source": "execution-time events of every conv launch of one untimed step, "
                                               "stream-time events around the same launches"}
        # north_star: HBM GB/s of the interp / loss kernels (and the BN passes) vs the peak,
        # live hipEvents over one untimed step right before the timed region
        out["hbm_kernels"] = hbm
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            aff = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            aff = os.cpu_count() or 1
        threads = min(aff, int(os.environ.get("OMP_NUM_THREADS", aff)))
        out["cpu_baseline"] = cpu_baseline(threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
