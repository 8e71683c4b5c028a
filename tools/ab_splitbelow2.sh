#!/bin/bash
# A/B after the data-gradient tile changes: fwd / data-grad K-split threshold (grids below
# ADAPTSEG_EXP_SPLITBELOW tiles split K; default 257).  Alternating runs.
set -e
mkdir -p gpurun_out
for cfg in c2 c3; do
  for rep in 1 2; do
    for sb in 257 129 513; do
      ADAPTSEG_EXP_SPLITBELOW=$sb timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_sb_${cfg}_${sb}_$rep.json 2> gpurun_out/ab_sb_${cfg}_${sb}_$rep.err
    done
  done
done
