#!/bin/bash
# round 4: conv3's backward on term images too (ADAPTSEG_X3_BWD_TERMS=3) — parity of the
# model-level / full-resolution step tests under it, then the A/B against mode 2 at c2 / c3.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
ADAPTSEG_X3_BWD_TERMS=3 timeout -k 10 600 python -u -m pytest tests/test_fullres_gpu.py -k "c2 or c3" tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r4h.log 2>&1 || { tail -30 gpurun_out/pytest_r4h.log; exit 3; }
tail -1 gpurun_out/pytest_r4h.log
CFGS="c2 c3" ROUNDS=2 bash experiments/ab_env.sh 'm2|ADAPTSEG_X3_BWD_TERMS=2|' 'm3|ADAPTSEG_X3_BWD_TERMS=3|' || exit 4
