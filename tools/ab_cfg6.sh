#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ab_base.log 2>&1 || exit 3
ADAPTSEG_EXP_CFG6=1 timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ab_cfg6.log 2>&1 || exit 4
