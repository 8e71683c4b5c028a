#!/bin/bash
# round 4: the fp32 LDS-transposed epilogue also for stride-2 parity-class data gradients and
# activation gradients (the discriminators' LeakyReLU' and DeeplabVGG's ReLU' data gradients;
# libadaptseg.so) vs the per-element path for them (libadaptseg_s2old.so = head): parity, then
# c2 / c3 / c4 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_epilogue_paths_gpu.py tests/test_conv_coverage.py tests/test_ops_gpu.py \
  tests/test_vgg.py tests/test_fullres_gpu.py tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4y.log 2>&1 || { tail -40 gpurun_out/pytest_r4y.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4y.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c2 c3 c4" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_s2old.so|" || exit 4
