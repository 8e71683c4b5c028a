#!/usr/bin/env python3
"""Per-step wall time and caching-allocator state of the bench workload (diagnostic).

    python tools/step_times.py --config c4 --steps 8
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    from adaptsegnet_amd import kernels as K
    from adaptsegnet_amd.model import DeeplabMulti, DeeplabVGG, FCDiscriminator
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    level, gan, batch, src, tgt, gen, math = bench.CONFIGS[args.config]
    K.set_conv_math(K.MATH_BF16 if math == "bf16" else K.MATH_F32X3)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1338)
    model = (DeeplabMulti if gen == "DeeplabMulti" else DeeplabVGG)(num_classes=19).to(dev).train()
    D1 = FCDiscriminator(num_classes=19).to(dev) if level == "multi-level" else None
    D2 = FCDiscriminator(num_classes=19).to(dev)
    tr = AdaptSegTrainer(model, D1, D2, StepConfig(level=level, gan=gan, input_size=src, input_size_target=tgt))
    g = torch.Generator().manual_seed(1338)
    xs = (torch.rand(batch, 3, src[1], src[0], generator=g) * 273.7 - 122.7).to(dev)
    lab = torch.randint(0, 19, (batch, src[1], src[0]), generator=g).to(dev)
    xt = (torch.rand(batch, 3, tgt[1], tgt[0], generator=g) * 273.7 - 122.7).to(dev)
    for i in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(i, [(xs, lab, xt)])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = torch.cuda.memory_stats(dev)
        print(f"step {i}: {dt * 1e3:8.1f} ms  allocated {st['allocated_bytes.all.current'] / 2**30:6.1f} GiB  "
              f"peak {st['allocated_bytes.all.peak'] / 2**30:6.1f}  reserved {st['reserved_bytes.all.current'] / 2**30:6.1f}  "
              f"alloc_retries {st.get('num_alloc_retries', 0)}  cuda_mallocs {st.get('segment.all.allocated', 0)}",
              flush=True)


if __name__ == "__main__":
    main()
