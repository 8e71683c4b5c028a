#!/bin/bash
# A/B: deferred weight-gradient joins inside the trainer step (ADAPTSEG_EXP_DEFERJOIN=1).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/dj_all.*
for r in 1 2; do
  for E in "X=0" "ADAPTSEG_EXP_DEFERJOIN=1"; do
    for cf in c2 c3; do
      env $E timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/dj_x.log 2>&1 || exit 3
      tail -1 gpurun_out/dj_x.log >> gpurun_out/dj_all.jsonl
      echo "$E $cf" >> gpurun_out/dj_all.tags
    done
  done
done
