#!/bin/bash
# A/B: data gradients on the occupancy-3 BK-16 tile (cfg 8) for every eligible product ("all"),
# for 1x1 products only ("1x1", the default), or never ("old", the BK-32 cfg-0 tile).  Alternating runs.
# Usage (GPU box): bash tools/ab_dgcfg.sh [configs...]
set -e
mkdir -p gpurun_out
cfgs=${@:-c2 c3}
for cfg in $cfgs; do
  for rep in 1 2; do
    ADAPTSEG_EXP_DG8_ALL=1 timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_dg_${cfg}_all_$rep.json 2> gpurun_out/ab_dg_${cfg}_all_$rep.err
    timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_dg_${cfg}_1x1_$rep.json 2> gpurun_out/ab_dg_${cfg}_1x1_$rep.err
    ADAPTSEG_EXP_DGCFG=0 timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_dg_${cfg}_old_$rep.json 2> gpurun_out/ab_dg_${cfg}_old_$rep.err
  done
done
