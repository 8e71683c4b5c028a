#!/bin/bash
# A/B: target-domain pass on a second stream (default) vs sequential; step parity tests.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_checkpoint.py tests/test_bf16_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ov_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ov_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ov_c2_on.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-overlap > gpurun_out/ov_c2_off.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/ov_c3_on.log 2>&1 || exit 5
timeout -k 10 600 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/ov_c5_on.log 2>&1 || exit 6
timeout -k 10 600 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --no-overlap > gpurun_out/ov_c5_off.log 2>&1 || exit 7
