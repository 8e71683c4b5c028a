#!/usr/bin/env python3
"""Per-launch HBM-side bytes of one kernel symbol from two rocprofv3 --pmc passes.

    python tools/traffic_summary.py gpurun_out/traffic_c2 "igemm_fast_kernel<0, 128, 128, 2, 2, 32, false, false, false>" > out.json

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts 64 B per 128-B memory-side
read request, i.e. half the bytes of a coalesced streaming read (MI355X_MICROARCH.md, HBM):
it is doubled here; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are L2 memory-side
(fabric) counters, so Infinity-Cache hits are included.
"""
import csv
import glob
import json
import sys

root, sym = sys.argv[1], sys.argv[2]


def mangled_key(name):
    """'k<1, 128, 256>' -> 'kILi1ELi128ELi256EE' ('false' -> Lb0E): rocprofv3 leaves symbols
    with bf16 (DF16b) parameters mangled, so an int / bool template is also matched in that form."""
    if "<" not in name:
        return None
    base, args = name.split("<", 1)
    parts = [a.strip() for a in args.rstrip(">").split(",")]
    enc = {"false": "Lb0E", "true": "Lb1E"}
    if not all(a.lstrip("-").isdigit() or a in enc for a in parts):
        return None
    return base + "I" + "".join(enc.get(a, f"Li{a}E") for a in parts) + "E"


MKEY = mangled_key(sym)


def per_launch(counter):
    vals = []
    for path in glob.glob(f"{root}/{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter and (sym in r["Kernel_Name"] or (MKEY and MKEY in r["Kernel_Name"])):
                vals.append(float(r["Counter_Value"]) * 1024.0)
    return sum(vals) / len(vals) if vals else None, len(vals)


fetch, nf = per_launch("FETCH_SIZE")
write, nw = per_launch("WRITE_SIZE")
out = {"kernel": sym, "launches": nf, "fetch_bytes_raw": fetch, "write_bytes": write,
       "fetch_bytes": None if fetch is None else 2.0 * fetch}
out["traffic_bytes_per_launch"] = (None if fetch is None or write is None
                                   else out["fetch_bytes"] + write)
print(json.dumps(out, indent=1))
