#!/bin/bash
# Round-5 evidence, final tree (second part): the default bench command (with the CPU baseline),
# kernel traces of c2-c5 and the HBM traffic passes of c5 (its weight-gradient kernel changed).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default_r5f.json 2> gpurun_out/bench_default_r5f.err || exit 5
tail -c 200 gpurun_out/bench_default_r5f.json
bash tools/gpu_prof.sh c5 r5f traffic || exit 6
bash tools/gpu_prof.sh c2 r5f || exit 7
bash tools/gpu_prof.sh c4 r5f || exit 8
bash tools/gpu_prof.sh c3 r5f || exit 9
echo EVIDENCE_F_OK
