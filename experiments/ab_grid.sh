#!/bin/bash
# bench arms on one box, alternating: bash experiments/ab_grid.sh "lib.so:flags lib2.so:flags ..." reps bench args...
# flags: "-" for none, or experiments/bench_variant.py switches joined by "," (e.g. --no-x3-copies)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
ARMS=$1; REPS=$2; shift 2
for rep in $(seq $REPS); do
for A in $ARMS; do
  L=${A%%:*}; F=${A#*:}; [ "$F" = "-" ] && F=""; F=${F//,/ }
  # shellcheck disable=SC2086
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u experiments/bench_variant.py $F --no-cpu-baseline "$@" > gpurun_out/abg.json 2>/dev/null || exit 4
  python -c "import json,sys; d=json.loads(open('gpurun_out/abg.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['config']['workload'][:3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" "$A"
done
done
