#!/bin/bash
# Round-5 evidence, final tree after the wide-Cout tile default: smoke(), the whole GPU suite,
# bench lines c2-c5 and the default command, and c4's kernel trace + traffic passes.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_r5d.log 2>&1 || { tail -20 gpurun_out/smoke_r5d.log; exit 3; }
tail -1 gpurun_out/smoke_r5d.log
bash tools/gpu_run.sh r5d "tests -m gpu" "c2 c3 c4 c5" || exit 4
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default_r5d.json 2> gpurun_out/bench_default_r5d.err || exit 5
tail -c 200 gpurun_out/bench_default_r5d.json
bash tools/gpu_prof.sh c4 r5d traffic || exit 6
echo EVIDENCE_D_OK
