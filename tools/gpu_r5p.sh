#!/bin/bash
# Round 5: DeeplabVGG term images only on the wide layers (ADAPTSEG_VGG_TERMS_MIN_C): parity, then
# c4 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_vgg.py -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_vgg.log 2>&1 || { tail -30 $O/pytest_vgg.log; exit 3; }
tail -1 $O/pytest_vgg.log
CFGS="c4" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 't0|ADAPTSEG_VGG_TERMS=0|' \
  't1c512|ADAPTSEG_VGG_TERMS=1 ADAPTSEG_VGG_TERMS_MIN_C=512|' 't2c512|ADAPTSEG_VGG_TERMS=2 ADAPTSEG_VGG_TERMS_MIN_C=512|' \
  't1c256|ADAPTSEG_VGG_TERMS=1 ADAPTSEG_VGG_TERMS_MIN_C=256|' 't2c256|ADAPTSEG_VGG_TERMS=2 ADAPTSEG_VGG_TERMS_MIN_C=256|' \
  't2c1024|ADAPTSEG_VGG_TERMS=2 ADAPTSEG_VGG_TERMS_MIN_C=1024|' > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5P_OK
