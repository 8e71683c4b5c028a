#!/bin/bash
# round 4: backward BN pass grids one at a time — the apply at 1024 blocks (bwa1024), the sums at
# 256 (bwr256); base 512 / 512.  Library builds differing only in those constants, c5 and c2.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
L=adaptsegnet_amd/lib
CFGS="c5 c2" ROUNDS=2 bash experiments/ab_env.sh 'base||' "bwa1024|ADAPTSEG_LIBRARY=$L/libadaptseg_bwa1024.so|" \
  "bwr256|ADAPTSEG_LIBRARY=$L/libadaptseg_bwr256.so|" || exit 4
