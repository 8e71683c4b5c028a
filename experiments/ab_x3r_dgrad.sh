#!/bin/bash
# F32X3: layer 3-4 conv2 data gradients on the term-image kernel too (BN2's backward writing dY2's
# terms; ADAPTSEG_X3R_DGRAD=1 during this A/B), c2 arms alternating
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
ADAPTSEG_X3R_DGRAD=1 timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_x3rdg.log 2>&1 || { tail -30 gpurun_out/pt_x3rdg.log; exit 3; }
tail -1 gpurun_out/pt_x3rdg.log
for CFG in c2 c3; do
for rep in 1 2; do
for v in 0 1; do
  ADAPTSEG_X3R_DGRAD=$v timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abx.json 2>gpurun_out/abx.err || { tail -5 gpurun_out/abx.err; exit 4; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abx.json').read().strip().splitlines()[-1]); print('x3r_dgrad', sys.argv[1], sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" "$v" "$CFG"
done
done
done
