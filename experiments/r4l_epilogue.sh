#!/bin/bash
# round 4: the conv epilogue's read-backs (residual + its bitmap, accumulate target) loaded per
# 8-row batch before use, 32-bit offsets (libadaptseg.so) vs the per-element read-back epilogue of
# the round-4 head (libadaptseg_epiold.so, same sources otherwise): parity of every conv product,
# then the A/B at c2 / c3 / c5 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_coverage.py tests/test_mask_bits_gpu.py tests/test_bn_bf16_storage_gpu.py \
  tests/test_ops_gpu.py tests/test_x3_terms_gpu.py tests/test_fullres_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4l.log 2>&1 || { tail -40 gpurun_out/pytest_r4l.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4l.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c2 c3 c5" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_epiold.so|" || exit 4
