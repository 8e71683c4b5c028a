#!/bin/bash
# Round-5 evidence, final tree (after the N >= 64 bf16 LDS-DMA threshold; D forward reuse, second-head-only step, bf16 weight-
# gradient pixel walk): smoke(), the whole GPU suite, bench lines c2-c5.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_r5g.log 2>&1 || { tail -20 gpurun_out/smoke_r5g.log; exit 3; }
tail -1 gpurun_out/smoke_r5g.log
bash tools/gpu_run.sh r5g "tests -m gpu" "c2 c3 c4 c5" || exit 4
echo EVIDENCE_G_OK
