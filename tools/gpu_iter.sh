#!/bin/bash
# Kernel iteration: all GPU parity tests (one process), then the per-shape conv bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-i}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/iter_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/iter_tests_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/conv_bench.py > gpurun_out/convbench_$TAG.log 2>&1
