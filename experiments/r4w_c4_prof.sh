#!/bin/bash
# round 4: kernel traces of c4 under the round-3 tree (_r3tree) and this tree, same box
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
mkdir -p $R/gpurun_out/c4cmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4cmp/r4 -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/c4cmp/r4.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4cmp/r3 -o run --output-format csv -- python3 $R/_r3tree/bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/c4cmp/r3.log 2>&1 || exit 4
echo done
