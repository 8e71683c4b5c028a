#!/bin/bash
# A/B of the weight-gradient split-K target (blocks per grid).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for t in ${WGTS:-1024 512 768 2048}; do
  ADAPTSEG_EXP_WGT=$t timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/wgt_$t.log 2>&1 || exit 3
done
