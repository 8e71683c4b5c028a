#!/bin/bash
# bf16 parity + c5 bench + c2 bench (regression) + rocprof of c5.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-c5}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_bf16_gpu.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/bf16_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/bf16_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2_$TAG.log 2>&1 || exit 5
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5_$TAG -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c5_$TAG.log 2>&1 || exit 6
