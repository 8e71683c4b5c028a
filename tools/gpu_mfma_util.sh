#!/bin/bash
# MFMA utilisation of the atrous convs (SURVEY 8(d) target >= 40 %): one --pmc pass per conv
# (no trace domains) over conv_bench restricted to that conv, all three ops.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mfma
cd /tmp
for FILT in l3.conv2 l4.conv2 aspp6 aspp5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/mfma/$FILT -o run --output-format csv -- python3 $R/tools/conv_bench.py --filter $FILT --reps 3 > $R/gpurun_out/mfma/$FILT.log 2>&1 || exit 3
done
