#!/bin/bash
# rocprofv3 kernel-trace stats of the c2 bench with and without the F32X3 operand copies
# (experiments/bench_variant.py): gpurun_out/prof_copies_{on,off}/
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
CFG=${1:-c2}
for V in on off; do
  A=""; [ $V = off ] && A="--no-x3-copies"
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_copies_$V -o run --output-format csv -- \
    python3 $R/experiments/bench_variant.py $A --config $CFG --steps 2 --warmup 1 --no-cpu-baseline \
    > $R/gpurun_out/prof_copies_$V.json 2> $R/gpurun_out/prof_copies_$V.err || exit 3
done
