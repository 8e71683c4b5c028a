#!/bin/bash
# Round-5 evidence, part C: atrous MFMA utilisation passes (F32X3 and bf16) and the c2 step's
# per-kernel counters (in the step vs alone).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
bash tools/gpu_mfma_util.sh f32x3 || exit 3
bash tools/gpu_mfma_util.sh bf16 || exit 4
bash tools/gpu_step_pmc.sh c2 || exit 5
echo EVIDENCE_C_OK
