#!/bin/bash
# Same-box A/B of the F32X3 operand copies: bench.py (copies on) vs experiments/bench_variant.py
# --no-x3-copies, alternating twice.  bash experiments/ab_copies.sh bench args...
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
for rep in 1 2; do
for V in "" "--no-x3-copies"; do
  timeout -k 10 300 python -u experiments/bench_variant.py $V --no-cpu-baseline "$@" > gpurun_out/abc.json 2>/dev/null || exit 4
  python -c "import json,sys; d=json.loads(open('gpurun_out/abc.json').read().strip().splitlines()[-1]); print(sys.argv[1] or 'copies', d['config']['workload'][:3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" "$V"
done
done
