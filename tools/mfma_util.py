#!/usr/bin/env python3
"""MFMA utilisation per kernel from rocprofv3 --pmc runs of tools/gpu_mfma_util.sh.

util = SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs),
per dispatch, averaged per (conv, kernel).  GRBM_GUI_ACTIVE is the sum over the 8 XCDs
(MI355X_MICROARCH.md, DVFS note), so GRBM/8 is the kernel's duration in shader cycles.

    python tools/mfma_util.py gpurun_out/mfma
"""
import collections
import csv
import os
import re
import sys

root = sys.argv[1]
print(f"{'conv':10s} {'kernel':62s} {'disp':>5s} {'MFMA util':>9s} {'eff. GHz':>8s}")
for filt in sorted(os.listdir(root)):
    path = os.path.join(root, filt, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        if "igemm" not in r["Kernel_Name"] and "tap" not in r["Kernel_Name"]:
            continue
        key = r["Dispatch_Id"]
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
        names[key] = re.sub(r"\(adaptseg::.*", "", r["Kernel_Name"].replace("void adaptseg::", ""))[:62]
        per[key]["_ns"] = float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0)
    agg = collections.defaultdict(list)
    for key, c in per.items():
        if c.get("GRBM_GUI_ACTIVE", 0) > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0
            util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
            ghz = cyc / c["_ns"] if c["_ns"] > 0 else 0.0
            agg[names[key]].append((util, ghz))
    for name, v in agg.items():
        u = sum(x[0] for x in v) / len(v)
        g = sum(x[1] for x in v) / len(v)
        print(f"{filt:10s} {name:62s} {len(v):5d} {u:9.3f} {g:8.2f}")
