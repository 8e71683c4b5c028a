#!/bin/bash
# round 4: fp32-output epilogue of the F32X3 kernels through a per-wave LDS transpose (16-B stores
# and read-backs; libadaptseg.so) vs the batched per-element epilogue of the round-4 head
# (libadaptseg_v4old.so): parity, then c2 / c3 (c5 as a control) on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_coverage.py tests/test_mask_bits_gpu.py tests/test_x3_terms_gpu.py \
  tests/test_ops_gpu.py tests/test_fullres_gpu.py tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4p.log 2>&1 || { tail -40 gpurun_out/pytest_r4p.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4p.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c2 c3 c5" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_v4old.so|" || exit 4
