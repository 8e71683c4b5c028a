#!/bin/bash
# Round 5: stream overlap of the two domains and of the discriminator step (StepConfig
# overlap_domains / overlap_d): bit-identity tests, then c2 / c3 / c5 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "overlap" > $O/pytest_overlap.log 2>&1 || { tail -30 $O/pytest_overlap.log; exit 3; }
tail -2 $O/pytest_overlap.log
CFGS="c2 c3 c5" ROUNDS=1 STEPS=10 bash experiments/ab_env.sh 'base||' 'ovdom||--overlap' 'ovd||--overlap-d' 'both||--overlap --overlap-d' > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 4; }
CFGS="c2" ROUNDS=1 STEPS=10 bash experiments/ab_env.sh 'base||' 'both||--overlap --overlap-d' >> $O/ab.txt 2>&1 || exit 5
cat $O/ab.txt
echo R5C_OK
