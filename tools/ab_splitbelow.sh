#!/bin/bash
# A/B: split-K for fwd / data-grad grids of up to one (257) or two (513, target 1024) blocks
# per CU.  ADAPTSEG_EXP_SPLITBELOW / ADAPTSEG_EXP_FDTARGET.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for cfg in "256 512" "257 512" "513 1024" "257 512" "513 1024"; do
  set -- $cfg
  for c in c3 c2; do
    ADAPTSEG_EXP_SPLITBELOW=$1 ADAPTSEG_EXP_FDTARGET=$2 timeout -k 10 300 python bench.py --config $c --steps 4 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/sb_${c}_$1_$2.log 2>&1 || exit 3
    tail -1 gpurun_out/sb_${c}_$1_$2.log >> gpurun_out/sb_all.jsonl
    echo "$c $1 $2" >> gpurun_out/sb_all.tags
  done
done
