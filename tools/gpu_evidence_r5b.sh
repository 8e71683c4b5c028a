#!/bin/bash
# Round-5 evidence, part B: final-tree kernel-trace summaries (tools/gpu_prof.sh) and HBM traffic
# passes (FETCH_SIZE / WRITE_SIZE, separate --pmc runs) for c2-c5 (or $CFGS).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
for C in ${CFGS:-c2 c3 c4 c5}; do
  bash tools/gpu_prof.sh $C r5 traffic || exit 3
  echo "$C done"
done
echo EVIDENCE_B_OK
