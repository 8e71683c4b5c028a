#!/bin/bash
# round 4: bf16-output epilogue of the LDS-DMA bf16 kernels through a per-wave LDS transpose (16-B
# stores and read-backs) with their BK-32 builds at 4 waves / SIMD (launch bounds) — libadaptseg.so
# — vs the round-4 head (libadaptseg_v8old.so): parity, then c5 (and c2 as a control) on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bn_bf16_storage_gpu.py tests/test_bf16_gpu.py tests/test_conv_coverage.py \
  tests/test_fullres_gpu.py tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4o.log 2>&1 || { tail -40 gpurun_out/pytest_r4o.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4o.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c5 c2" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_v8old.so|" || exit 4
