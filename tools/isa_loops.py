#!/usr/bin/env python3
"""Instruction mix of every MFMA loop in a device assembly dump (hipcc -S --cuda-device-only).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -S --cuda-device-only -o /tmp/k.s adaptsegnet_amd/csrc/X.hip
    python tools/isa_loops.py /tmp/k.s [symbol-substring ...]

Per kernel and per backward-branch loop that holds MFMAs: MFMAs, VALU (non-MFMA v_*), SALU,
LDS (ds_*), global/buffer instructions, s_waitcnt and barriers in the body, plus the kernel's
VGPR count and scratch size — the static side of the step_pmc.py VALU/MFMA ratio.
"""
import re
import sys

src = open(sys.argv[1]).read()
want = sys.argv[2:]
head = re.compile(r"^(_Z\w+):", re.M)
starts = [(m.start(), m.group(1)) for m in head.finditer(src)]
for n, (pos, name) in enumerate(starts):
    if want and not any(w in name for w in want):
        continue
    end = starts[n + 1][0] if n + 1 < len(starts) else len(src)
    lines = src[pos:end].split("\n")
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    meta = src[src.find(".name:           " + name):] if ".name:           " + name in src else ""
    vg = re.search(r"\.vgpr_count:\s+(\d+)", src[src.find(name + ":"):]) if False else None
    sgpr = re.search(r";\s*NumVgprs:\s*(\d+)", src[pos:end])
    scratch = re.search(r";\s*ScratchSize:\s*(\d+)", src[pos:end])
    print(f"{name}  vgpr {sgpr.group(1) if sgpr else '?'}  scratch {scratch.group(1) if scratch else '?'}")
    for i, l in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
        if not m:
            continue
        t = m.group(1) or m.group(2)
        if t not in labels or labels[t] >= i:
            continue
        body = [x.strip() for x in lines[labels[t]:i + 1]]
        body = [x for x in body if x and not x.startswith((";", ".")) and not x.endswith(":")]
        ins = [x.split()[0] for x in body]
        mf = sum(1 for x in ins if x.startswith("v_mfma"))
        if not mf:
            continue
        valu = [x for x in ins if x.startswith("v_") and not x.startswith("v_mfma")]
        cnt = {}
        for x in valu:
            cnt[x] = cnt.get(x, 0) + 1
        top = ", ".join(f"{k} {v}" for k, v in sorted(cnt.items(), key=lambda kv: -kv[1])[:8])
        print(f"  loop {t:12s} {len(ins):4d} ins: mfma {mf:3d} valu {len(valu):4d} "
              f"salu {sum(1 for x in ins if x.startswith('s_')):4d} ds {sum(1 for x in ins if x.startswith('ds_')):3d} "
              f"vmem {sum(1 for x in ins if x.startswith(('global_', 'buffer_'))):3d} "
              f"wait {sum(1 for x in ins if x == 's_waitcnt'):3d} bar {sum(1 for x in ins if x == 's_barrier'):2d}")
        print(f"      {top}")
