#!/bin/bash
# A/B of two library builds on one box: bash experiments/ab_lib.sh A.so CONFIG "pytest selection"
#   A = adaptsegnet_amd/lib/libadaptseg_a.so (the previous build), B = the in-tree build.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
A=${1:-adaptsegnet_amd/lib/libadaptseg_a.so}
CFG=${2:-c5}
SEL=${3:-none}
if [ "$SEL" != "none" ]; then
  # shellcheck disable=SC2086
  timeout -k 10 600 python -u -m pytest $SEL -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/abl_t.log 2>&1 || { tail -5 gpurun_out/abl_t.log; exit 3; }
  tail -1 gpurun_out/abl_t.log
fi
for rep in 1 2 3; do
  ADAPTSEG_LIBRARY=$A timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl.json 2>/dev/null || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/abl.json').read().strip().splitlines()[-1]); print('A', round(d['value'],3), round(d['ms_per_step'],2))"
  timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl.json 2>/dev/null || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/abl.json').read().strip().splitlines()[-1]); print('B', round(d['value'],3), round(d['ms_per_step'],2))"
done
