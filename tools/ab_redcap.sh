#!/bin/bash
# A/B of the split-K reduce grid cap (ADAPTSEG_EXP_REDCAP).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/redcap_all.*
for r in 1 2; do
  for t in ${REDS:-8192 1024 512}; do
    for cf in c2 c3; do
      ADAPTSEG_EXP_REDCAP=$t timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/redcap_x.log 2>&1 || exit 3
      tail -1 gpurun_out/redcap_x.log >> gpurun_out/redcap_all.jsonl
      echo "$t $cf" >> gpurun_out/redcap_all.tags
    done
  done
done
