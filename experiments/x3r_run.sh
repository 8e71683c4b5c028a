#!/bin/bash
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -k "presplit or f32x3_accuracy or unbiased or deterministic" -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_x3r.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_x3r.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3_presplit > gpurun_out/cs_x3r.txt 2>&1 || exit 5
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 > gpurun_out/cs_x3.txt 2>&1 || exit 6
tail -4 gpurun_out/cs_x3r.txt; tail -4 gpurun_out/cs_x3.txt
