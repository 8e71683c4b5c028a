#!/bin/bash
# bench.py over several library builds, alternating: bash experiments/ab_many.sh "libA libB ..." reps bench args...
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
LIBS=$1; REPS=$2; shift 2
for rep in $(seq $REPS); do
for L in $LIBS; do
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/abm.json 2>/dev/null || exit 4
  python -c "import json,sys; d=json.loads(open('gpurun_out/abm.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['config']['workload'][:3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" $L
done
done
