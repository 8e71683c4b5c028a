#!/bin/bash
# A/B of the weight-gradient split target (blocks per grid, rounded down) on c2 / c3.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/wgt2_all.*
for r in 1 2; do
  for t in 512 768 1024 384; do
    for cf in c2 c3; do
      ADAPTSEG_EXP_WGT=$t timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/wgt2_x.log 2>&1 || exit 3
      tail -1 gpurun_out/wgt2_x.log >> gpurun_out/wgt2_all.jsonl
      echo "$t $cf" >> gpurun_out/wgt2_all.tags
    done
  done
done
