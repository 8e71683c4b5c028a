#!/bin/bash
# Round-5 evidence, part A: smoke(), the whole GPU test suite, bench lines c2-c5 (10 steps after 3
# warm-up) and the default bench command with its CPU-baseline leg.  Each step under its own limit.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_r5.log 2>&1 || { tail -20 gpurun_out/smoke_r5.log; exit 3; }
tail -1 gpurun_out/smoke_r5.log
bash tools/gpu_run.sh r5 "tests -m gpu" "c2 c3 c4 c5" || exit 4
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default_r5.json 2> gpurun_out/bench_default_r5.err || exit 5
tail -c 300 gpurun_out/bench_default_r5.json
echo EVIDENCE_A_OK
