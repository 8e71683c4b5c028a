#!/bin/bash
# A/B the default library vs adaptsegnet_amd/lib/libadaptseg_ab.so on bench.py (args passed on),
# alternating twice.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
for rep in 1 2; do
for L in adaptsegnet_amd/lib/libadaptseg.so adaptsegnet_amd/lib/libadaptseg_ab.so; do
  timeout -k 10 300 python -u tools/dbg/with_lib.py $L bench.py --no-cpu-baseline --no-roofline "$@" > gpurun_out/abb.json 2>/dev/null || exit 4
  python -c "import json,sys; d=json.loads(open('gpurun_out/abb.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['config']['workload'][:3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" $L
done
done
