#!/bin/bash
# A/B: forward-only tile variant (ADAPTSEG_EXP_FWDCFG 8 = BK16 occupancy 3, 6 = BK16).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
rm -f gpurun_out/cfg3_all.*
for r in 1 2; do
  for c in def 8 6; do
    for cf in c2 c3; do
      if [ $c = def ]; then E=""; else E="ADAPTSEG_EXP_FWDCFG=$c"; fi
      env $E timeout -k 10 300 python bench.py --config $cf --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/cfg3_${c}_${cf}.log 2>&1 || exit 3
      tail -1 gpurun_out/cfg3_${c}_${cf}.log >> gpurun_out/cfg3_all.jsonl
      echo "$c $cf" >> gpurun_out/cfg3_all.tags
    done
  done
done
