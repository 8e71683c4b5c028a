#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/p4_all.*
for r in 1 2; do
  for E in "X=0" "ADAPTSEG_EXP_HIPRIO=0"; do
    for cf in c4 c5; do
      env $E timeout -k 10 300 python bench.py --config $cf --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p4_x.log 2>&1 || exit 3
      tail -1 gpurun_out/p4_x.log >> gpurun_out/p4_all.jsonl
      echo "$E $cf" >> gpurun_out/p4_all.tags
    done
  done
done
