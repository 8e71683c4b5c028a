#!/bin/bash
# A/B: step on a high-priority stream (weight gradients on a normal-priority side stream).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/prio_all.*
for r in 1 2; do
  for E in "X=0" "ADAPTSEG_EXP_HIPRIO=1"; do
    for cf in c2 c3; do
      env $E timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/prio_x.log 2>&1 || exit 3
      tail -1 gpurun_out/prio_x.log >> gpurun_out/prio_all.jsonl
      echo "$E $cf" >> gpurun_out/prio_all.tags
    done
  done
done
