#!/bin/bash
# Round 5: bf16 conv math, thin conv inputs (stem Cin 3, D.conv1 Cin 19) padded to 8 channels for
# their weight gradients (the LDS-DMA weight-gradient kernel) instead of 4: parity, c5 arms.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_bf16_gpu.py tests/test_bn_bf16_storage_gpu.py "tests/test_fullres_gpu.py" -k "bf16 or c5" \
  -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
CFGS="c5" ROUNDS=3 STEPS=10 bash experiments/ab_env.sh 'pad4|ADAPTSEG_WGRAD_PAD8=0|' 'pad8|ADAPTSEG_WGRAD_PAD8=1|' | tee $O/ab.txt || exit 4
echo R5AF_OK
