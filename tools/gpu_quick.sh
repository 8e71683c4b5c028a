#!/bin/bash
# Quick GPU iteration: op + bf16 tests, then c2 and c5 benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_data.py tests/test_ops_gpu.py tests/test_bf16_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/quick_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/quick_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2_$TAG.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.log 2>&1 || exit 5
