#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-i5}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bf16_gpu.py tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/it5_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/it5_tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/it5_cb_$TAG.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/it5_c2_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/it5_c5_$TAG.log 2>&1 || exit 5
