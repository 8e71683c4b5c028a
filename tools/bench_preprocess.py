#!/usr/bin/env python3
"""Throughput of the GPU input pipeline (adaptseg_gta5_preprocess) on GTA5-sized batches.

    python tools/bench_preprocess.py [--batch 4] [--steps 20]

One step = one batch of decoded 1914x1052 RGB images + uint8 id labels -> the reference's
1280x720 float32 BGR-mean CHW images and int64 trainId labels (dataset/gta5_dataset.py:54-68),
already resident in HBM.  roofline: HBM-bound; algorithmic bytes per image = the compulsory
input (H*W*3 + H*W) and output (3*h*w*4 + h*w*8) bytes, against 8 TB/s.  cpu_baseline: the
reference's own per-item path (Pillow resize + numpy remap / BGR / mean, as
tests/golden/gen_data_golden.py restates it) on one core — the work each of the reference's
4 DataLoader workers (train:35) does per image.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    from adaptsegnet_amd import data
    dev = torch.device("cuda", 0)
    H, W, (ow, oh) = 1052, 1914, (1280, 720)
    rng = np.random.default_rng(0)
    imgs_np = rng.integers(0, 256, (args.batch, H, W, 3), dtype=np.uint8)
    labs_np = rng.integers(0, 34, (args.batch, H, W), dtype=np.uint8)
    imgs, labs = torch.from_numpy(imgs_np).to(dev), torch.from_numpy(labs_np).to(dev)
    for _ in range(3):
        data.preprocess(imgs, labs, (ow, oh))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        data.preprocess(imgs, labs, (ow, oh))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    per_img = H * W * 3 + H * W + 3 * oh * ow * 4 + oh * ow * 8
    ach = per_img * args.batch / (ms / 1e3) / 1e9
    out = {"metric": "GTA5 preprocess images/sec (1914x1052 -> 1280x720, image + label)",
           "value": args.batch / (ms / 1e3), "unit": "images/s", "ms_per_step": ms, "batch": args.batch,
           "roofline": {"bound": "hbm", "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0,
                        "algorithmic_bytes_per_image": per_img}}
    if not args.no_cpu_baseline:
        from gen_data_golden import item
        torch.set_num_threads(1)
        t0 = time.perf_counter()
        k = 3
        for i in range(k):
            item(imgs_np[i % args.batch], labs_np[i % args.batch], (ow, oh))
        dt = (time.perf_counter() - t0) / k
        out["cpu_baseline"] = {"value": 1.0 / dt, "unit": "images/s", "cores": 1, "kind": "port",
                               "sample": f"{k} items of the reference's __getitem__ arithmetic (Pillow resize + "
                                         f"numpy remap/BGR/mean), {dt * 1e3:.0f} ms each"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
