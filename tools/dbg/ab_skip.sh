#!/bin/bash
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/skip_t.log 2>&1; tail -2 gpurun_out/skip_t.log
for rep in 1 2; do
  timeout -k 10 300 python -u tools/dbg/no_skip.py bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abs.json 2>/dev/null || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]); print('noskip', round(d['value'],3), round(d['ms_per_step'],2))"
  timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abs.json 2>/dev/null || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]); print('skip', round(d['value'],3), round(d['ms_per_step'],2))"
done
