#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel (short names) over the dispatches of a run.

    python tools/pmc_summary.py gpurun_out/pmc_TAG/s*/run_counter_collection.csv [--match igemm]
"""
import collections
import csv
import re
import sys

args = sys.argv[1:]
match = ""
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1]
    del args[i:i + 2]
paths = args
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for p in paths:
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"]
        if match and match not in name:
            continue
        short = re.sub(r"\(adaptseg::ConvParams\)", "", name.replace("void adaptseg::", ""))[:70]
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
