#!/bin/bash
# Thin convs: parity (ops, warper, model), then the c2 and warper benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_warper_gpu.py > gpurun_out/thin_ops.log 2>&1 || exit 2
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py > gpurun_out/thin_model.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/thin_b.log 2>&1 || exit 4
timeout -k 10 300 python tools/bench_warper.py --no-cpu-baseline > gpurun_out/thin_w.log 2>&1 || exit 5
