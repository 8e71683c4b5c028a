#!/bin/bash
# A/B of the 128x128 tile config against ADAPTSEG_EXP_CFG=<cfg> on the per-shape conv bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ab_base.log 2>&1 || exit 3
for c in "$@"; do
  ADAPTSEG_EXP_CFG=$c timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ab_cfg$c.log 2>&1 || exit 4
done
