#!/usr/bin/env python3
"""Kernels of one bench step in the step vs alone, with their counters (tools/gpu_step_pmc.sh).

The kernel-trace pass times every launch of the step with the weight-gradient stream beside it;
rocprofv3 serialises dispatches while it collects counters, so the --pmc passes over the same
step time each launch alone, with its counters.  Per kernel symbol and grid shape: launches,
in-step and alone duration, MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x
1024 SIMDs)), VALU busy (SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024), quad-cycles),
the wave-time split (issue-stalled SQ_WAIT_INST_ANY, parked SQ_WAIT_ANY, issuing
SQ_ACTIVE_INST_ANY, each / SQ_WAVE_CYCLES), VALU and LDS instructions per MFMA, LDS bank
conflicts per LDS-array cycle, and the L2 memory-side traffic per launch (FETCH_SIZE x 2 +
WRITE_SIZE).

    python tools/step_pmc.py gpurun_out/step_pmc_c2 "igemm_x3_kernel<2, false>" "igemm_x3_kernel<1, false>" ...
"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
KEYS = sys.argv[2:]


def mangled(name):
    """'k<1, 128>' -> 'kILi1ELi128E' (rocprofv3 leaves templates with bf16 parameters mangled)."""
    if "<" not in name:
        return None
    base, args = name.split("<", 1)
    parts = [a.strip() for a in args.rstrip(">").split(",")]
    enc = {"false": "Lb0E", "true": "Lb1E"}
    if not all(a.lstrip("-").isdigit() or a in enc for a in parts):
        return None
    return base + "I" + "".join(enc.get(a, f"Li{a}E") for a in parts)


def key_of(name):
    for k in KEYS:
        m = mangled(k)
        if k in name or (m and m in name):
            return k
    return None


def grid(r):
    """total work-items of the dispatch (the trace gives X / Y / Z, the counter CSV the product)"""
    if r.get("Grid_Size_X"):
        return str(int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1))
    return r.get("Grid_Size") or "?"


trace = collections.defaultdict(list)
for path in glob.glob(f"{root}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        k = key_of(r["Kernel_Name"])
        if k:
            trace[(k, grid(r))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

alone = collections.defaultdict(lambda: collections.defaultdict(dict))
for path in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    p = path[len(root):].strip("/").split("/")[0]
    for r in csv.DictReader(open(path)):
        k = key_of(r["Kernel_Name"])
        if not k:
            continue
        d = alone[(k, grid(r))][(p, r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["_us"] = (float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)) / 1e3


def mean(v):
    v = list(v)
    return sum(v) / len(v) if v else float("nan")


def per(ds, f):
    out = []
    for d in ds:
        try:
            out.append(f(d))
        except (KeyError, ZeroDivisionError):
            pass
    return mean(out)


print(f"{'kernel':44s} {'grid':>9s} {'n':>3s} {'step us':>8s} {'alone us':>8s} {'MFMA':>6s} {'VALU':>6s} "
      f"{'stall':>6s} {'parked':>6s} {'issue':>6s} {'valu/mf':>7s} {'lds/mf':>6s} {'bankc':>6s} {'MB/launch':>9s}")
for (k, g) in sorted(set(trace) | set(alone), key=lambda kg: (kg[0], int(kg[1]) if kg[1].isdigit() else 0)):
    st = trace.get((k, g), [])
    ds = list(alone.get((k, g), {}).values())
    al = mean(d["_us"] for d in ds if d.get("_us", 0) > 0)
    simd = lambda d: d["GRBM_GUI_ACTIVE"] / 8 * 1024   # noqa: E731
    mf = per(ds, lambda d: d["SQ_VALU_MFMA_BUSY_CYCLES"] / simd(d))
    vb = per(ds, lambda d: 4 * d["SQ_ACTIVE_INST_VALU"] / simd(d))
    wi = per(ds, lambda d: d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"])
    wa = per(ds, lambda d: d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"])
    ai = per(ds, lambda d: d["SQ_ACTIVE_INST_ANY"] / d["SQ_WAVE_CYCLES"])
    vpm = per(ds, lambda d: d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"])
    lpm = per(ds, lambda d: d["SQ_INSTS_LDS"] / d["SQ_INSTS_MFMA"])
    bc = per(ds, lambda d: d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"])
    fe = per(ds, lambda d: 2 * 1024 * d["FETCH_SIZE"])
    wr = per(ds, lambda d: 1024 * d["WRITE_SIZE"])
    print(f"{k[:44]:44s} {g:>9s} {len(st):3d} {mean(st):8.1f} {al:8.1f} {mf:6.3f} {vb:6.3f} {wi:6.3f} {wa:6.3f} "
          f"{ai:6.3f} {vpm:7.2f} {lpm:6.2f} {bc:6.3f} {(fe + wr) / 1e6:9.1f}")
