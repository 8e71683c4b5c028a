#!/bin/bash
# Round-4 evidence refresh after the last epilogue change: the c2 / c5 kernel-trace summaries,
# then the whole GPU suite, smoke(), bench lines c2-c5 and the default command (tools/gpu_evidence_r4b.sh).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
bash tools/gpu_prof.sh c2 r4c || exit 3
bash tools/gpu_prof.sh c5 r4c || exit 4
bash tools/gpu_evidence_r4b.sh || exit 5
