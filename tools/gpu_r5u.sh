#!/bin/bash
# Round 5: s_setprio(1) around the MFMA cluster of the bf16 LDS-DMA kernel's K step (the guide's
# 8-phase template) — experiment build (EXTRA=-DADAPTSEG_G16_SETPRIO=1) vs in-tree, c5 alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5u
mkdir -p $O
for rep in 1 2 3; do
  for L in libadaptseg.so libadaptseg_sp.so; do
    ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 \
      --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 4; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('ab c5', sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', [(k['selector'], round(k['frac'],3)) for k in r['by_kernel']], flush=True)" $O/b.json $L | tee -a $O/ab.txt
  done
done
echo R5U_OK
