#!/bin/bash
# A/B of the per-shape conv bench under an env override, with extra conv_bench args:
#   ab_env2.sh TAG "conv_bench args" NAME VALUE...
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
TAG=$1; ARGS=$2; V=$3; shift 3
timeout -k 10 300 python tools/conv_bench.py $ARGS > gpurun_out/ab_${TAG}_base.log 2>&1 || exit 3
for x in "$@"; do
  env $V=$x timeout -k 10 300 python tools/conv_bench.py $ARGS > gpurun_out/ab_${TAG}_${V}_$x.log 2>&1 || exit 4
done
