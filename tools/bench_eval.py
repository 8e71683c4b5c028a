#!/usr/bin/env python3
"""Evaluation throughput: evaluate_cityscapes.py's per-image body.

    python tools/bench_eval.py [--batch 1] [--steps 10] [--warmup 2]

One step = eval-mode DeeplabMulti forward on a 1024x512 image, interp of output2 to
1024x2048 + argmax (one fused kernel), and the confusion-matrix update against a uint8
label-id map (compute_iou.fast_hist).  Prints ONE JSON line; ``roofline`` is for the fused
upsample+argmax kernel (HBM-bound: algorithmic bytes = the 1/8-scale logits read once +
one byte per output pixel), timed with HIP events on its stream.  ``cpu_baseline`` = the
oracle (stock-PyTorch CPU fp32 eval forward + interp + argmax + numpy fast_hist) for 1 image.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    from adaptsegnet_amd.evaluate import ConfusionMatrix, predict, upsample_argmax
    from adaptsegnet_amd.model import DeeplabMulti
    dev = torch.device("cuda", 0)
    torch.manual_seed(1338)
    model = DeeplabMulti(num_classes=19).to(dev)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(args.batch, 3, 512, 1024, generator=g) * 273.7 - 122.7).to(dev)
    gt = torch.randint(0, 34, (args.batch, 1024, 2048), generator=g, dtype=torch.uint8).to(dev)
    cm = ConfusionMatrix(19, device=dev)
    for _ in range(args.warmup):
        cm.update(gt, predict(model, x))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cm.update(gt, predict(model, x))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the fused kernel alone, on the model's 1/8-scale map (input-size upsample as model(image))
    logits = model(x)[1].detach()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        upsample_argmax(logits, (1024, 2048))
    e1.record()
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1) / reps
    n, c, h, w = logits.shape
    alg_bytes = n * h * w * c * 4 + n * 1024 * 2048
    gbs = alg_bytes / (k_ms * 1e-3) / 1e9
    out = {"metric": "eval images/s (1024x512 -> 1024x2048 prediction + confusion update), DeeplabMulti",
           "value": args.batch * args.steps / dt, "unit": "images/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
           "dtype": "f32", "data": "synthetic", "config": {"workload": "eval, batch %d" % args.batch},
           "miou_of_random_model": cm.miou(),
           "roofline": {"bound": "hbm", "kernel": "upsample_argmax_kernel", "achieved": gbs,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": k_ms,
                        "traffic": None,
                        "note": "input-size logits (model(image) upsamples to 512x1024 first)"}}
    if not args.no_cpu_baseline:
        from oracle import reference_eval as E
        from oracle import reference_torch as R
        threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "64")))
        torch.set_num_threads(threads)
        G = R.to_torch(R.det_state(R.g_specs(), 1338), dtype=torch.float32)
        xc = x[:1].cpu()
        gtc = gt[:1].cpu().numpy()
        t0 = time.perf_counter()
        with torch.no_grad():
            _, p2 = R.g_forward(G, xc, (1024, 512), train=False)
            pred, _ = E.predict_argmax(p2.float(), (1024, 2048))
        from adaptsegnet_amd.evaluate import CITYSCAPES_TRAIN_IDS
        mapping = [(i, CITYSCAPES_TRAIN_IDS.get(i, 255)) for i in range(34)]
        E.fast_hist(E.label_mapping(gtc, mapping), pred.numpy(), 19)
        ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 1.0 / ct, "unit": "images/s", "cores": threads, "kind": "port",
                               "sample": f"1 image eval (oracle eval forward + interp + argmax + fast_hist); {ct:.2f} s"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
