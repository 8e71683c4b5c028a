#!/bin/bash
# F32X3 weight-gradient split rounding (ADAPTSEG_X3_WGRAD_ROUND_NEAREST / _TARGET): per-shape
# (tools/conv_bench.py, atrous convs) and the c2 / c3 step, arms alternating on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for L in libadaptseg.so libadaptseg_rn.so libadaptseg_t512.so; do
  for F in l3.conv2 l4.conv2; do
    ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 200 python -u tools/conv_bench.py --math f32x3 --filter $F 2>&1 | grep -E "^$F +2 " | sed "s/^/$L /" || exit 3
  done
done
bash experiments/ab_grid.sh "libadaptseg.so:- libadaptseg_rn.so:- libadaptseg_t512.so:-" 2 --config c2 --steps 10 --warmup 3
