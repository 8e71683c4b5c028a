#!/usr/bin/env python3
"""RCCL process group with a high-priority stream (the bench.py option) initialises and
all-reduces on one GPU (world size 1): a smoke check of the N > 1 init path."""
import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29541")
torch.cuda.set_device(0)
opts = dist.ProcessGroupNCCL.Options(); opts.is_high_priority_stream = True
dist.init_process_group("nccl", world_size=1, rank=0, device_id=torch.device("cuda", 0), pg_options=opts)
t = torch.ones(1024, device="cuda")
w = dist.all_reduce(t, async_op=True); w.wait(); torch.cuda.synchronize()
print("nccl hp pg ok", float(t.sum()))
dist.destroy_process_group()
