#!/bin/bash
# rocprofv3 kernel trace + stats of one bench config (no PMC).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${1:-c3}
mkdir -p $R/gpurun_out
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$CFG -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$CFG.log 2>&1
