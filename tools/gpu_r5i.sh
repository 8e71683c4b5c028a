#!/bin/bash
# Round 5: BN backward sums fused into the data-gradient epilogue (ADAPTSEG_BN_SUMS): op parity,
# the model / full-resolution step parity, then c2 / c3 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "fused_bn_sums or dgrad_into_bn or batchnorm or conv_fwd_dgrad_wgrad or epilogues" > $O/pytest_ops.log 2>&1 \
  || { tail -30 $O/pytest_ops.log; exit 3; }
tail -2 $O/pytest_ops.log
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_fullres_gpu.py -x -q --timeout 600 \
  --timeout-method thread -k "not bench_batch" > $O/pytest_model.log 2>&1 || { tail -30 $O/pytest_model.log; exit 4; }
tail -2 $O/pytest_model.log
CFGS="c2 c3" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 'sums|ADAPTSEG_BN_SUMS=1|' 'nosums|ADAPTSEG_BN_SUMS=0|' \
  > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5I_OK
