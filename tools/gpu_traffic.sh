#!/bin/bash
# HBM-side traffic of the bench's kernels: two separate --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over the same bench command, no trace domains.  Summarised by tools/traffic_summary.py.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${1:-c2}
OUT=$R/gpurun_out/traffic_$CFG
mkdir -p $OUT
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d $OUT/$C -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/$C.log 2>&1 || exit 3
done
