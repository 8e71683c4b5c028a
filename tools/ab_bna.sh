#!/bin/bash
# A/B of the BN apply passes' block target (ADAPTSEG_EXP_BNA).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/bna_all.*
for r in 1 2; do
  for t in ${BNAS:-512 256 2048}; do
    for cf in c2 c3; do
      ADAPTSEG_EXP_BNA=$t timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/bna_x.log 2>&1 || exit 3
      tail -1 gpurun_out/bna_x.log >> gpurun_out/bna_all.jsonl
      echo "$t $cf" >> gpurun_out/bna_all.tags
    done
  done
done
