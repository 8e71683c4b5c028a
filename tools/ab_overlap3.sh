#!/bin/bash
# A/B: domain overlap (target pass on a side stream) with the high-priority main chain.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/ov3_all.*
for r in 1 2; do
  for O in "" "--overlap"; do
    for cf in c2 c3; do
      timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline $O > gpurun_out/ov3_x.log 2>&1 || exit 3
      tail -1 gpurun_out/ov3_x.log >> gpurun_out/ov3_all.jsonl
      echo "ov=$O $cf" >> gpurun_out/ov3_all.tags
    done
  done
done
