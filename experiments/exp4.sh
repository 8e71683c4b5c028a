#!/bin/bash
# fp32-packed B for the F32X3 kernel (libB = current build) vs bf16-term-packed B (libA): parity, per-shape, c2
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_ops_gpu.py > gpurun_out/exp4_tests.txt 2>&1 || { tail -30 gpurun_out/exp4_tests.txt; exit 3; }
tail -2 gpurun_out/exp4_tests.txt
bash experiments/ab_libs.sh "libA.so libB.so" --math f32x3 --filter l3.conv2 || exit 4
bash experiments/ab_libs.sh "libA.so libB.so" --math f32x3 --filter l4.conv2 || exit 4
bash experiments/ab_bench_many.sh "libA.so libB.so" --steps 10 --warmup 3 || exit 5
