#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV: top kernels, per-step time."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'ms/step':>9} {'%':>5} {'calls/step':>10} {'avg us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:9.2f} {float(r['Percentage']):5.1f} "
          f"{float(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:9.1f}  {r['Name'][:100]}")
print(f"total kernel time per step: {tot / 1e6 / steps:.2f} ms")
