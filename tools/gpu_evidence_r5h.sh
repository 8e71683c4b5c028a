#!/bin/bash
# Round-5 evidence, final tree (second part, after the N >= 64 bf16 threshold): the default bench
# command with its CPU baseline, and the c5 / c2 kernel traces.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default_r5h.json 2> gpurun_out/bench_default_r5h.err || exit 5
tail -c 200 gpurun_out/bench_default_r5h.json
bash tools/gpu_prof.sh c5 r5h || exit 6
bash tools/gpu_prof.sh c2 r5h || exit 7
echo EVIDENCE_H_OK
