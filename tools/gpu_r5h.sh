#!/bin/bash
# Round 5: kernel-time summary + traffic passes of the c2 step on the current tree, and the c5
# step's counters in the step vs alone (the bf16 BN passes / LDS-DMA kernels).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
bash tools/gpu_prof.sh c2 r5 traffic || exit 3
bash tools/gpu_step_pmc.sh c5 || exit 4
echo R5H_OK
