#!/bin/bash
# MFMA utilisation of the atrous convs (SURVEY 8(d) target >= 40 %): one --pmc pass per conv
# (no trace domains) over conv_bench restricted to that conv, all three ops.
#   bash tools/gpu_mfma_util.sh [conv math: f32 | f32x3 | bf16] [tag] [extra conv_bench args]
#   (default f32x3, the library default; e.g. bf16 c5 "--width 1280 --height 720": c5's source geometry)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MATH=${1:-f32x3}
TAG=${2:-$MATH}
EXTRA=${3:-}
OUT=$R/gpurun_out/mfma_$TAG
mkdir -p $OUT
cd /tmp
for FILT in l3.conv2 l4.conv2 aspp6 aspp5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/$FILT -o run --output-format csv -- python3 $R/tools/conv_bench.py --filter $FILT --reps 3 --math $MATH $EXTRA > $OUT/$FILT.log 2>&1 || exit 3
done
