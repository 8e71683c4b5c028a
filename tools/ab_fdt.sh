#!/bin/bash
# A/B of the fwd / data-grad split target for grids of <= 256 tiles (ADAPTSEG_EXP_FDTARGET).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/fdt_all.*
for r in 1 2; do
  for t in 512 768 1024; do
    for cf in c3 c5; do
      ADAPTSEG_EXP_FDTARGET=$t timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/fdt_x.log 2>&1 || exit 3
      tail -1 gpurun_out/fdt_x.log >> gpurun_out/fdt_all.jsonl
      echo "$t $cf" >> gpurun_out/fdt_all.tags
    done
  done
done
