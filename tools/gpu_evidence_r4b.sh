#!/bin/bash
# Round-4 evidence, part B: the whole GPU test suite, smoke(), bench lines c2-c5 (10 steps after 3
# warm-up) and the default bench command with its CPU-baseline leg.  Each step under its own limit.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_r4.log 2>&1 || { tail -20 gpurun_out/smoke_r4.log; exit 3; }
bash tools/gpu_run.sh r4 "tests -m gpu" "c2 c3 c4 c5" || exit 4
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default_r4.json 2> gpurun_out/bench_default_r4.err || exit 5
tail -c 400 gpurun_out/bench_default_r4.json
echo EVIDENCE_B_OK
