#!/bin/bash
# Round-4 final-tree kernel-trace summaries for c2-c5 (tools/gpu_prof.sh, no PMC passes).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
for C in c2 c3 c4 c5; do
  bash tools/gpu_prof.sh $C r4d || exit 3
  echo "$C done"
done
