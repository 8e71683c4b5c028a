#!/bin/bash
# rocprofv3 kernel-trace stats of one bench config on several library builds:
#   bash experiments/ab_prof.sh TAG CONFIG "libA libB ..."   -> gpurun_out/prof_TAG_<lib>/
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
TAG=$1; CFG=$2; LIBS=$3
for L in $LIBS; do
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_${L%.so} \
    -o run -- python3 bench.py --config "$CFG" --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}_${L%.so}.log 2>&1 || exit 4
done
