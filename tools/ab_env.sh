#!/bin/bash
# A/B of the per-shape conv bench under an environment override: ab_env.sh NAME VALUE...
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
V=$1; shift
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ab_base.log 2>&1 || exit 3
for x in "$@"; do
  env $V=$x timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ab_${V}_$x.log 2>&1 || exit 4
done
