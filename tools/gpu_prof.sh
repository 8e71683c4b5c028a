#!/bin/bash
# rocprofv3 kernel-trace stats of one bench command, then the HBM traffic passes
# (FETCH_SIZE / WRITE_SIZE, separate --pmc runs, no trace domains).
#   bash tools/gpu_prof.sh CFG TAG [traffic]
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${1:-c2}
TAG=${2:-r2}
OUT=$R/gpurun_out/prof_${CFG}_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 3
if [ "$3" = "traffic" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C -d $OUT/$C -o run --output-format csv -- \
      python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/$C.log 2>&1 || exit 4
  done
fi
