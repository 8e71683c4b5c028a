#!/bin/bash
# Cost of the live roofline timing: c2 with the roofline (dominant kernel events only in the
# timed region) vs --no-roofline, alternated.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rt_on_$r.log 2>&1 || exit 3
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/rt_off_$r.log 2>&1 || exit 3
done
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/rt_c3.log 2>&1 || exit 3
