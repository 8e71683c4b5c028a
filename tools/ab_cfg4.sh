#!/bin/bash
# A/B: data-gradient tile (ADAPTSEG_EXP_DGCFG=6: BK16, LDS 34 KB -> 4 blocks/CU) and 1x1
# weight-gradient tile (ADAPTSEG_EXP_WGCFG=6 / 8) vs the defaults.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/cfg4_all.*
for r in 1 2; do
  for E in "X=0" "ADAPTSEG_EXP_DGCFG=6" "ADAPTSEG_EXP_WGCFG=6" "ADAPTSEG_EXP_WGCFG=8"; do
    for cf in c2 c3; do
      env $E timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/cfg4_x.log 2>&1 || exit 3
      tail -1 gpurun_out/cfg4_x.log >> gpurun_out/cfg4_all.jsonl
      echo "$E $cf" >> gpurun_out/cfg4_all.tags
    done
  done
done
