#!/bin/bash
# round 4: split-K reduce with its read-back operands issued before the slab loads
# (libadaptseg.so) vs loaded after the slab sum (libadaptseg_rdold.so, the round-4 head's
# conv_igemm.hip, same sources otherwise): parity, then the A/B at c2 / c3 / c5 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_coverage.py tests/test_bn_bf16_storage_gpu.py tests/test_ops_gpu.py \
  tests/test_fullres_gpu.py tests/test_checkpoint.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4m.log 2>&1 || { tail -40 gpurun_out/pytest_r4m.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4m.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c2 c3 c5" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_rdold.so|" || exit 4
