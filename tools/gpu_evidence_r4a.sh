#!/bin/bash
# Round-4 evidence, part A (profiles first, so the bench lines of part B carry this tree's PMC
# traffic): rocprofv3 kernel-trace summaries + FETCH/WRITE traffic passes of the c2 / c3 / c5
# bench, and the atrous MFMA-utilisation passes under both conv maths.  Each step under its own
# limit; stops at the first failure.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for CFG in c2 c3 c5; do
  bash tools/gpu_prof.sh $CFG r4 traffic || exit 3
  echo "prof $CFG ok"
done
bash tools/gpu_mfma_util.sh f32x3 || exit 4
bash tools/gpu_mfma_util.sh bf16 || exit 5
echo EVIDENCE_A_OK
