#!/bin/bash
# A/B: BN backward sums fused into the data-gradient epilogue vs the separate reduction pass.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
ADAPTSEG_BNSUMS=1 timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_fused.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_unfused.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_fused2.log 2>&1 || exit 5
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ab -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_ab.log 2>&1 || exit 6
