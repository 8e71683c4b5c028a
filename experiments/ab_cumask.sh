#!/bin/bash
# Weight-gradient stream confined to a fraction of the CUs (engine._side_stream,
# ADAPTSEG_WGRAD_CU_FRACTION), arms alternating on one box:  bash experiments/ab_cumask.sh CFG "0 0.5 0.75" REPS
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
CFG=${1:-c2}; FR=${2:-"0 0.5 0.75"}; REPS=${3:-2}
for rep in $(seq $REPS); do
for f in $FR; do
  if [ "$f" = "0" ]; then unset ADAPTSEG_WGRAD_CU_FRACTION; else export ADAPTSEG_WGRAD_CU_FRACTION=$f; fi
  timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abm.json 2>gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 4; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abm.json').read().strip().splitlines()[-1]); print('frac', sys.argv[1], sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" "$f" "$CFG"
done
done
unset ADAPTSEG_WGRAD_CU_FRACTION
