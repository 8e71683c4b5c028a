#!/bin/bash
# round 4: the general (per-element) epilogue path — stride-2 parity scatter, activation gradients,
# partial tiles — with its read-backs issued per 4-row batch (libadaptseg.so) vs per element
# (libadaptseg_genold.so = the round-4 head): parity, then c2 / c3 / c5 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_coverage.py tests/test_ops_gpu.py tests/test_fullres_gpu.py \
  tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4r.log 2>&1 || { tail -40 gpurun_out/pytest_r4r.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4r.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c2 c3 c5" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_genold.so|" || exit 4
# the stem's forward on channel-padded operands (engine.PAD_STEM) vs the per-element fp32 kernel
CFGS="c2 c5" ROUNDS=2 bash experiments/ab_env.sh 'stem4|ADAPTSEG_PAD_STEM=1|' 'stem3|ADAPTSEG_PAD_STEM=0|' || exit 5
