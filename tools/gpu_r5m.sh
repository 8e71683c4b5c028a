#!/bin/bash
# Round 5: the target forward enqueued before the source backward (StepConfig.target_first):
# bit-identity tests, then c2 / c3 / c5 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 400 --timeout-method thread -k "overlap" \
  > $O/pytest_overlap.log 2>&1 || { tail -30 $O/pytest_overlap.log; exit 3; }
tail -1 $O/pytest_overlap.log
CFGS="c2 c3 c5" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 'seq||' 'tfirst||--target-first' > $O/ab.txt 2>&1 \
  || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5M_OK
