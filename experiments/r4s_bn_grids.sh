#!/bin/bash
# round 4: BN pass grid sizes — the forward apply at 1024 / 2048 blocks (it runs without the
# weight-gradient stream beside it; base 512), the backward passes at 1024 (base 512) — library
# builds differing only in those constants, c5 and c2 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
L=adaptsegnet_amd/lib
CFGS="c5 c2" ROUNDS=2 bash experiments/ab_env.sh 'base||' "fa1024|ADAPTSEG_LIBRARY=$L/libadaptseg_fa1024.so|" \
  "fa2048|ADAPTSEG_LIBRARY=$L/libadaptseg_fa2048.so|" "bw1024|ADAPTSEG_LIBRARY=$L/libadaptseg_bw1024.so|" || exit 4
