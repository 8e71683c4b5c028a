#!/bin/bash
# round 4: the fp32 LDS-transposed epilogue also for forwards with a bias (DeeplabVGG's convs,
# the discriminators', the ASPP heads; libadaptseg.so) vs bias-carrying forwards on the
# per-element path (libadaptseg_nobias.so = head): parity, then c4 / c2 / c5 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_coverage.py tests/test_ops_gpu.py tests/test_vgg.py tests/test_fullres_gpu.py \
  tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4t.log 2>&1 || { tail -40 gpurun_out/pytest_r4t.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4t.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c4 c2 c5" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_nobias.so|" || exit 4
