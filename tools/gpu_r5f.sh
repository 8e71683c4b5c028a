#!/bin/bash
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5f
mkdir -p $O
ADAPTSEG_VGG_TERMS=2 timeout -k 10 300 python -u tools/step_times.py --config c4 --steps 6 > $O/t2_steps.txt 2>&1 || exit 3
ADAPTSEG_VGG_TERMS=0 timeout -k 10 300 python -u tools/step_times.py --config c4 --steps 6 > $O/t0_steps.txt 2>&1 || exit 4
cat $O/t2_steps.txt $O/t0_steps.txt
