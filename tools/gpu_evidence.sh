#!/bin/bash
# End-of-round evidence in one GPU session: GPU tests, bench lines c2..c5, the default bench
# line (with the CPU baseline), per-shape conv tables, c2 kernel trace + dominant-kernel traffic.
# Each step under its own limit; stops at the first failure.
export TMPDIR=/tmp
TAG=${1:-r2}
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
bash tools/gpu_run.sh $TAG "tests -m gpu" "c2 c3 c4 c5" || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err || exit 5
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 > gpurun_out/conv_shapes_$TAG.txt 2>&1 || exit 6
timeout -k 10 300 python -u tools/conv_bench.py --math bf16 > gpurun_out/conv_shapes_bf16_$TAG.txt 2>&1 || exit 7
bash tools/gpu_prof.sh c2 $TAG traffic || exit 8
echo EVIDENCE_OK
