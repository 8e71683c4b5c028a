#!/bin/bash
# round 4: split-K targets of the weight gradients re-tuned on the round-4 program (library builds
# differing only in the target: bf16 LDS-DMA 256 (base) / 128 / 384 at c5; F32X3 staged 384 (base) /
# 256 / 512 at c2), one box, arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
L=adaptsegnet_amd/lib
CFGS="c5" ROUNDS=2 bash experiments/ab_env.sh 'base||' "g128|ADAPTSEG_LIBRARY=$L/libadaptseg_g128.so|" "g384|ADAPTSEG_LIBRARY=$L/libadaptseg_g384.so|" || exit 3
CFGS="c2" ROUNDS=2 bash experiments/ab_env.sh 'base||' "x256|ADAPTSEG_LIBRARY=$L/libadaptseg_x256.so|" "x512|ADAPTSEG_LIBRARY=$L/libadaptseg_x512.so|" || exit 4
