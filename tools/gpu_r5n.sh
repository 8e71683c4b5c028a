#!/bin/bash
# Round 5 diagnostic: what bounds the bf16 LDS-DMA forward / data-gradient kernel on layer-3/4
# shapes — timing-only builds (numerically meaningless) whose A rows (1), B rows (2), both (3) all
# read one L2-resident 128-B line, or that issue no LDS-DMA at all (4).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5n
mkdir -p $O
for L in libadaptseg.so libadaptseg_dbg1.so libadaptseg_dbg2.so libadaptseg_dbg3.so libadaptseg_dbg4.so; do
  echo "== $L"
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 200 python -u tools/conv_bench.py --math bf16 --reps 10 \
    --filter "l3.conv" > $O/$L.l3.txt 2>&1 || { tail -5 $O/$L.l3.txt; exit 3; }
  grep -E "^l3" $O/$L.l3.txt | grep -v " 2 "
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 200 python -u tools/conv_bench.py --math bf16 --reps 10 \
    --filter "l4.conv2" > $O/$L.l4.txt 2>&1 || { tail -5 $O/$L.l4.txt; exit 4; }
  grep -E "^l4" $O/$L.l4.txt | grep -v " 2 "
done
echo R5N_OK
