#!/bin/bash
# Round 5: DeeplabVGG (c4) with the two domains on two streams, re-measured after the D forward reuse.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out/r5ae
CFGS="c4" ROUNDS=3 STEPS=10 bash experiments/ab_env.sh 'seq||' 'ov||--overlap on' | tee gpurun_out/r5ae/ab.txt || exit 4
echo R5AE_OK
