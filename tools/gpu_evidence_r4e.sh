#!/bin/bash
# Round-4 final-tree HBM traffic passes (FETCH_SIZE, WRITE_SIZE; separate --pmc runs) for c2, c3, c5 (or $CFGS).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
for C in ${CFGS:-c2 c3 c5}; do
  bash tools/gpu_traffic.sh $C || exit 3
  echo "$C done"
done
