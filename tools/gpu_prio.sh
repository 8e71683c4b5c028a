#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-p}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k conv > gpurun_out/prio_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/prio_tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/prio_cb_$TAG.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prio_c2_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python tools/conv_bench.py --math bf16 > gpurun_out/prio_cb16_$TAG.log 2>&1 || exit 5
