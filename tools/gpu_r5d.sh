#!/bin/bash
# Round 5: DeeplabVGG (c4) on F32X3 term images (engine.VGG_TERMS 0 / 1 / 2): parity, then the c4
# line per mode, arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vgg.py -x -q --timeout 300 --timeout-method thread > $O/pytest_vgg.log 2>&1 || { tail -30 $O/pytest_vgg.log; exit 3; }
tail -2 $O/pytest_vgg.log
CFGS="c4" ROUNDS=2 STEPS=8 bash experiments/ab_env.sh 't0|ADAPTSEG_VGG_TERMS=0|' 't0ov|ADAPTSEG_VGG_TERMS=0|--overlap' 't1|ADAPTSEG_VGG_TERMS=1|' 't2|ADAPTSEG_VGG_TERMS=2|' > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 4; }
cat $O/ab.txt
echo R5D_OK
