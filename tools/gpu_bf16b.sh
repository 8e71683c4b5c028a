#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-b}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bf16_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/b16_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/b16_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py --math bf16 > gpurun_out/b16cb256_$TAG.log 2>&1 || exit 3
ADAPTSEG_BF16_BN128=1 timeout -k 10 300 python tools/conv_bench.py --math bf16 > gpurun_out/b16cb128_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b16c5_256_$TAG.log 2>&1 || exit 5
ADAPTSEG_BF16_BN128=1 timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/b16c5_128_$TAG.log 2>&1 || exit 6
