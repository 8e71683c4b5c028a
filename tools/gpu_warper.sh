#!/bin/bash
# Warper measurement: bench_warper (with the CPU baseline) and a rocprofv3 kernel trace of it.
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-w1}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 600 python3 -u tools/bench_warper.py > gpurun_out/bench_warper_$TAG.json 2> gpurun_out/bench_warper_$TAG.err || exit 3
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_warper_$TAG -o run --output-format csv -- python3 $R/tools/bench_warper.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_warper_$TAG.log 2>&1 || exit 5
