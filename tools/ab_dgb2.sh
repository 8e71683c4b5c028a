#!/bin/bash
# A/B: stride-1 3x3 data gradients (cfg 0, BK 32) from the min-blocks-2 build ("b2", default:
# no fused BN-sum epilogue, accumulators in VGPRs, no SGPR spills) vs the min-blocks-1 build
# ("b1", ADAPTSEG_EXP_DGB1).  Alternating runs.  Usage (GPU box): bash tools/ab_dgb2.sh [configs...]
set -e
mkdir -p gpurun_out
cfgs=${@:-c2 c3}
for cfg in $cfgs; do
  for rep in 1 2; do
    timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_b2_${cfg}_b2_$rep.json 2> gpurun_out/ab_b2_${cfg}_b2_$rep.err
    ADAPTSEG_EXP_DGB1=1 timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ab_b2_${cfg}_b1_$rep.json 2> gpurun_out/ab_b2_${cfg}_b1_$rep.err
  done
done
