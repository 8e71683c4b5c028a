#!/usr/bin/env python3
"""The c5 bf16 data gradients in the step vs alone (experiments/r4n_c5_dgrad_pmc.sh).

The kernel-trace pass times every launch of the c5 step with the weight-gradient stream beside
it; rocprofv3 serialises dispatches while it collects counters, so the --pmc passes over the same
step time each launch alone, with its counters.  Per kernel and grid shape: in-step and alone
duration, MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)), the
fraction of wave time waiting on anything / on LDS, and the L2 memory-side fetch per launch.

    python tools/c5_dgrad_pmc.py gpurun_out/c5pmc
"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
KEYS = {"194": "igemm_bf16g_kernelILi1ELi128ELi256ELi32ELb0E", "194w": "igemm_bf16g_kernelILi1ELi256ELi128ELi32ELb0E",
        "94": "igemm_bf16g_kernelILi0ELi128ELi256ELi32ELb0E", "298": "igemm_bf16g_wgrad_kernelILi256E"}


def key_of(name):
    for k, m in KEYS.items():
        if m in name:
            return k
    return None


def grid(r):
    return r.get("Grid_Size_X") or r.get("Grid_Size") or "?"


trace = collections.defaultdict(list)
for path in glob.glob(f"{root}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        k = key_of(r["Kernel_Name"])
        if k:
            trace[(k, grid(r))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

alone = collections.defaultdict(lambda: collections.defaultdict(dict))
for p in ("p1", "p2", "p3"):
    for path in glob.glob(f"{root}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = key_of(r["Kernel_Name"])
            if not k:
                continue
            d = alone[(k, grid(r))][(p, r["Dispatch_Id"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["_us"] = (float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)) / 1e3


def mean(v):
    return sum(v) / len(v) if v else float("nan")


print(f"{'sel':5s} {'grid':>9s} {'n':>3s} {'step us':>8s} {'alone us':>8s} {'x':>5s} {'MFMA':>6s} {'wait':>6s} "
      f"{'LDSwait':>7s} {'MB/launch':>9s}")
for (k, g) in sorted(set(trace) | set(alone)):
    st = trace.get((k, g), [])
    disp = alone.get((k, g), {})
    p1 = [d for (p, _), d in disp.items() if p == "p1"]
    p2 = [d for (p, _), d in disp.items() if p == "p2"]
    p3 = [d for (p, _), d in disp.items() if p == "p3"]
    al = mean([d["_us"] for d in p1 if d.get("_us", 0) > 0])
    mf = mean([d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024) for d in p1
               if d.get("GRBM_GUI_ACTIVE")])
    wt = mean([d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"] for d in p1 if d.get("SQ_WAVE_CYCLES")])
    lw = mean([d["SQ_WAIT_INST_LDS"] / max(1.0, d.get("SQ_INSTS_LDS", 1.0)) for d in p2 if "SQ_WAIT_INST_LDS" in d])
    fs = mean([2 * 1024 * d["FETCH_SIZE"] / 1e6 for d in p3 if "FETCH_SIZE" in d])
    s = mean(st)
    print(f"{k:5s} {g:>9s} {len(st):3d} {s:8.1f} {al:8.1f} {s / al if al == al and al else float('nan'):5.2f} "
          f"{mf:6.3f} {wt:6.3f} {lw:7.1f} {fs:9.1f}")
