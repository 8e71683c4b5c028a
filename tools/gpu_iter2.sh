#!/bin/bash
# op tests, conv bench base vs cfg 8 (occupancy-3 BK16 tile), c2 bench (hbm kernels).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-i2}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/it_ops_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/it_ops_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/it_cb_base_$TAG.log 2>&1 || exit 3
ADAPTSEG_EXP_CFG=8 timeout -k 10 300 python tools/conv_bench.py > gpurun_out/it_cb_cfg8_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/it_c2_$TAG.log 2>&1 || exit 5
ADAPTSEG_EXP_CFG=8 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/it_c2cfg8_$TAG.log 2>&1 || exit 6
