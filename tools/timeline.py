#!/usr/bin/env python3
"""Busy/idle/concurrency analysis of a rocprofv3 kernel trace over a time window.

    python tools/timeline.py run_kernel_trace.csv [--last-fraction 0.33]

Reports, for the last fraction of the trace (the final timed step of a short bench run):
wall time, GPU-busy time (union of kernel intervals), time with >= 2 kernels in flight, and
busy time per stream and per kernel class on the critical (main) stream.
"""
import csv
import sys

path = sys.argv[1]
frac = float(sys.argv[sys.argv.index("--last-fraction") + 1]) if "--last-fraction" in sys.argv else 0.33
rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
ev.sort()
t0, t1 = ev[0][0], max(e[1] for e in ev)
cut = t1 - (t1 - t0) * frac
win = [e for e in ev if e[0] >= cut]
ws, we = win[0][0], max(e[1] for e in win)
points = sorted([(s, 1) for s, _, _, _ in win] + [(e, -1) for _, e, _, _ in win])
busy = conc = 0
depth, last = 0, ws
for t, d in points:
    if depth >= 1:
        busy += t - last
    if depth >= 2:
        conc += t - last
    depth += d
    last = t
print(f"window {(we - ws) / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms ({busy / (we - ws):.1%}), "
      f">=2 kernels {conc / 1e6:.2f} ms, kernels {len(win)}")
per = {}
for s, e, st, _ in win:
    per[st] = per.get(st, 0) + (e - s)
for st, v in sorted(per.items()):
    print(f"  stream {st}: kernel time {v / 1e6:.2f} ms")
