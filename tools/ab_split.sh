#!/bin/bash
# A/B of split-K rounding (floor, the default, vs ceil): per-shape conv timing + c2 bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/split_floor_cb.log 2>&1 || exit 3
ADAPTSEG_EXP_SPLITCEIL=1 timeout -k 10 300 python tools/conv_bench.py > gpurun_out/split_ceil_cb.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/split_floor_b.log 2>&1 || exit 4
ADAPTSEG_EXP_SPLITCEIL=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/split_ceil_b.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/split_floor_b2.log 2>&1 || exit 4
