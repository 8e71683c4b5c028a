#!/usr/bin/env python3
"""Warper throughput: the reference's default training mode.

    python tools/bench_warper.py [--batch 4] [--steps 5] [--warmup 2]

One step = one SOURCE_ONLY iteration with the warper on (train_gta2cityscapes_multi.py:259-286,
the script's default: SOURCE_ONLY = True, --warper default True): Warper forward on the
1024x512 source batch, DeeplabMulti forward, both heads warped by the field, cross-entropy on
the second, backward through the generator AND the warper (its parameters accumulate
gradients, as in the reference), generator SGD.  Synthetic inputs resident in HBM, random-init
weights.  Prints ONE JSON line with the step rate, the same step without the warper (its
cost), the warper's own forward+backward time, live HBM rooflines of the warp-specific kernels
(``hbm_kernels``: algorithmic bytes / summed launch time, HIP events on their stream), and
``cpu_baseline`` = the oracle (oracle/reference_warper.source_only_step, stock PyTorch CPU fp32)
for one batch-1 iteration on this host's cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
HBM_PEAK_GBS = 8000.0
WARP_IDS = (1008, 1009, 1010, 1011, 1012)


def timed(fn, steps, warmup):
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(warmup + i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / max(steps, 1)


def cpu_baseline(threads):
    from oracle import reference_torch as R
    from oracle import reference_warper as RW
    torch.set_num_threads(threads)
    G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=torch.float32, trainable=R.g_trainable)
    W = R.to_torch(R.det_state(RW.warper_specs(), 3001, conv_std=0.02), dtype=torch.float32,
                   trainable=RW.warper_trainable)
    D2 = R.to_torch(R.det_state(R.d_specs(), 2002), dtype=torch.float32, trainable=lambda k: True)
    opt, _, _ = R.make_optimizers(G, None, D2, R.DEFAULT_CFG)
    x = torch.from_numpy(R.det_images((1, 3, 512, 1024), 1)).float()
    lab = torch.from_numpy(R.det_labels((1, 512, 1024), 2))
    t0 = time.perf_counter()
    RW.source_only_step(G, W, opt, {"input_size": (1024, 512)}, 0, [(x, lab)])
    dt = time.perf_counter() - t0
    return {"value": 1.0 / dt, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": "1 source-only iteration with the warper (oracle/reference_warper.py, stock "
                      f"PyTorch CPU fp32), batch 1, 1024x512; {dt:.2f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, Warper
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    dev = torch.device("cuda", 0)
    torch.manual_seed(1338)
    model = DeeplabMulti(num_classes=19).to(dev)
    warper = Warper().to(dev)
    model.train()
    warper.train()
    n = args.batch
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(n, 3, 512, 1024, generator=g) * 273.7 - 122.7).to(dev)
    lab = torch.randint(0, 19, (n, 512, 1024), generator=g)
    lab[torch.rand(n, 512, 1024, generator=g) < 0.1] = 255
    lab = lab.to(dev)
    cfg = StepConfig(level="source-only", input_size=(1024, 512))
    tr = AdaptSegTrainer(model, None, None, cfg, warper=warper)
    tr_plain = AdaptSegTrainer(model, None, None, cfg)

    def step(i):
        tr.step(i, [(x, lab)])

    def step_plain(i):
        tr_plain.step(i, [(x, lab)])

    def warper_only(i):
        flow, _ = warper(x)
        flow.backward(torch.ones_like(flow))

    # warm everything, then time the warper step with the HBM kernel clocks on
    timed(step, 0, args.warmup)
    K.timing_enable_mem(True)
    dt = timed(step, args.steps, 0)
    K.timing_enable_mem(False)
    hbm = []
    for kid in WARP_IDS:
        ms_, by_, n_ = K.timing_read_id(kid)
        if n_:
            gbs = by_ / (ms_ / 1e3) / 1e9
            hbm.append({"kernel": K.MEM_KERNELS[kid], "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": by_ / n_,
                        "avg_launch_ms": ms_ / n_, "launches_per_step": n_ / args.steps})
    dt_plain = timed(step_plain, args.steps, 1)
    dt_w = timed(warper_only, args.steps, 1)
    # warper conv FLOPs per image (fwd + data-grad + weight-grad of every conv it runs)
    enc, out_conv = warper.encoder_blocks()
    dec, last = warper.decoder_blocks()
    fl, h, w = 0.0, 512, 1024
    convs = [(c, h, w) for c in [enc[0][0]]]
    ch, cw = enc[0][0].geom().out_hw(h, w)
    for conv, _ in enc[1:]:
        convs.append((conv, ch, cw))
        ch, cw = conv.geom().out_hw(ch, cw)
    convs.append((out_conv, ch, cw))
    ch, cw = out_conv.geom().out_hw(ch, cw)
    for conv, _ in dec:
        ch, cw = 2 * ch, 2 * cw
        convs.append((conv, ch, cw))
    convs.append((last, 2 * ch, 2 * cw))
    fwd = sum(c.geom().flops(n, hh, ww) for c, hh, ww in convs)
    bwd = fwd * 2 - convs[0][0].geom().flops(n, h, w)     # no data gradient into the images
    out = {
        "metric": "source-only train images/sec with the warper at 1024x512 (the reference's default mode)",
        "value": n / dt, "unit": "images/s", "ms_per_step": dt * 1e3, "batch": n, "dtype": "f32",
        "data": "synthetic (U[-122.7,151] pixels, uniform labels, 10% ignore=255), random-init weights",
        "without_warper": {"value": n / dt_plain, "ms_per_step": dt_plain * 1e3},
        "warper_fwd_bwd_ms": dt_w * 1e3,
        "warper_conv_gflop_per_image_fwd": fwd / n / 1e9,
        "warper_conv_tflops_achieved": (fwd + bwd) / dt_w / 1e12,
        "hbm_kernels": hbm,
    }
    if not args.no_cpu_baseline:
        try:
            aff = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            aff = os.cpu_count() or 1
        out["cpu_baseline"] = cpu_baseline(min(aff, int(os.environ.get("OMP_NUM_THREADS", aff))))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
