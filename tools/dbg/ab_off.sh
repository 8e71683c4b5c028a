#!/bin/bash
# A/B of one engine predicate on c5: bash tools/dbg/ab_off.sh NAME  (see patch_off.py)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
NAME=${1:-_copy_pays}
for rep in 1 2 3; do
  timeout -k 10 300 python -u tools/dbg/patch_off.py $NAME bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abo.json 2>/dev/null || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/abo.json').read().strip().splitlines()[-1]); print('off', round(d['value'],3), round(d['ms_per_step'],2))"
  timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abo.json 2>/dev/null || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/abo.json').read().strip().splitlines()[-1]); print('on ', round(d['value'],3), round(d['ms_per_step'],2))"
done
