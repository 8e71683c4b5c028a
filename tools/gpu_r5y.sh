#!/bin/bash
# Round 5: the single-level step computes only DeeplabMulti's second head (StepConfig.second_head_only):
# bit-identity / oracle parity, then interleaved c2 arms with and without it.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_fullres_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
CFGS="c2" ROUNDS=3 STEPS=10 bash experiments/ab_env.sh 'one||' 'both||--both-heads' | tee $O/ab.txt || exit 4
echo R5Y_OK
