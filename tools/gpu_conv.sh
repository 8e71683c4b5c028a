#!/bin/bash
# Kernel-iteration round: op parity tests + per-shape conv timing.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-c}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -q -p no:cacheprovider -x > gpurun_out/ops_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ops_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/conv_bench.py > gpurun_out/convbench_$TAG.log 2>&1
