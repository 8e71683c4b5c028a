#!/bin/bash
# round 4: mask-bitmap parity (new kernels first, then the model-level suites), then the A/B
# of engine.MASK_BITS and engine.HI_REDUCE at c2 / c5 (one box, arms alternating).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mask_bits_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_r4e_bits.log 2>&1 || { tail -30 gpurun_out/pytest_r4e_bits.log; exit 3; }
tail -1 gpurun_out/pytest_r4e_bits.log
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_fullres_gpu.py tests/test_bf16_gpu.py tests/test_ops_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r4e.log 2>&1
tail -3 gpurun_out/pytest_r4e.log
CFGS="c2 c5" ROUNDS=2 bash experiments/ab_env.sh 'bits_hi|ADAPTSEG_MASK_BITS=1 ADAPTSEG_HI_REDUCE=1|' 'nobits_hi|ADAPTSEG_MASK_BITS=0 ADAPTSEG_HI_REDUCE=1|' 'bits_lo|ADAPTSEG_MASK_BITS=1 ADAPTSEG_HI_REDUCE=0|' || exit 6
