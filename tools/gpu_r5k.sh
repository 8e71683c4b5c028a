#!/bin/bash
# Round 5: fused BN sums per BN (ADAPTSEG_BN_SUMS bit 1 = BN2 / conv3 data gradient, bit 2 = BN1 /
# conv2 data gradient), c2 and c3 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5k
mkdir -p $O
CFGS="c2 c3" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 'none|ADAPTSEG_BN_SUMS=0|' 'bn2|ADAPTSEG_BN_SUMS=1|' \
  'bn1|ADAPTSEG_BN_SUMS=2|' 'both|ADAPTSEG_BN_SUMS=3|' > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5K_OK
