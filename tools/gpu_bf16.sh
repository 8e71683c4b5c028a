#!/bin/bash
# bf16 conv path: its parity tests, the fp32 op tests (shared epilogue), per-shape timings.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-b}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/bf16_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ops_$TAG.log 2>&1 || exit 3
timeout -k 10 300 python tools/conv_bench.py --math bf16 > gpurun_out/convbench_bf16_$TAG.log 2>&1 || exit 4
