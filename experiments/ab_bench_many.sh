#!/bin/bash
# bench.py over several library builds (round robin, twice): bash experiments/ab_bench_many.sh "libA libB ..." bench args...
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
LIBS=$1; shift
for rep in 1 2; do
for L in $LIBS; do
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/abb.json 2>/dev/null || exit 4
  python -c "import json,sys; d=json.loads(open('gpurun_out/abb.json').read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[1], d['config']['workload'][:3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms frac', r.get('frac'))" $L
done
done
