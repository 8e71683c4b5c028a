#!/usr/bin/env python3
"""Host-side cost of one c2 step: wall time of trainer.step() returning (no sync) vs the GPU
time per step, to see whether the launch stream can run ahead of the GPU."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    from adaptsegnet_amd.model import DeeplabMulti, FCDiscriminator
    from adaptsegnet_amd.train import AdaptSegTrainer, StepConfig
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m, d2 = DeeplabMulti(19).to(dev), FCDiscriminator(19).to(dev)
    m.train()
    tr = AdaptSegTrainer(m, None, d2, StepConfig(level="single-level", input_size=(1024, 512),
                                                 input_size_target=(1024, 512)))
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(4, 3, 512, 1024, generator=g) * 273 - 122).to(dev)
    xt = (torch.rand(4, 3, 512, 1024, generator=g) * 273 - 122).to(dev)
    lab = torch.randint(0, 19, (4, 512, 1024), generator=g).to(dev)
    for i in range(2):
        tr.step(i, [(x, lab, xt)])
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for i in range(6):
        a = time.perf_counter()
        tr.step(2 + i, [(x, lab, xt)])
        host.append(time.perf_counter() - a)
    h_end = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print("host ms/step", [round(h * 1e3, 1) for h in host], "host total %.1f ms, wall %.1f ms (%.1f ms/step)"
          % (h_end * 1e3, wall * 1e3, wall / 6 * 1e3))


if __name__ == "__main__":
    main()
