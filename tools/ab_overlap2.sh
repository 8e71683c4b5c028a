#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --overlap > gpurun_out/ov2_on_$r.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ov2_off_$r.log 2>&1 || exit 4
done
