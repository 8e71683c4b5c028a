#!/bin/bash
# Round 5: conv3's backward on term images (ADAPTSEG_X3_BWD_TERMS=3) re-tested under the raised
# x3r weight-gradient split cap: parity under mode 3, then interleaved c2 / c3 arms.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5w
mkdir -p $O
ADAPTSEG_X3_BWD_TERMS=3 timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_fullres_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/pytest_m3.log 2>&1 || { tail -30 $O/pytest_m3.log; exit 3; }
tail -1 $O/pytest_m3.log
CFGS="c2 c3" ROUNDS=3 STEPS=10 bash experiments/ab_env.sh 'm2|ADAPTSEG_X3_BWD_TERMS=2|' 'm3|ADAPTSEG_X3_BWD_TERMS=3|' \
  | tee $O/ab.txt || exit 4
echo R5W_OK
