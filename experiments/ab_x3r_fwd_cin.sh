#!/bin/bash
# (historical: the ADAPTSEG_X3R_FWD / _MIN_CIN env switches it sets were removed from engine.py after
# the A/B; results in profiles/r3/x3r_forward_ab.txt)
# engine.x3_forward_terms threshold: conv2 forwards with Cin >= 256 (layers 3-4) vs >= 64 (all)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for rep in 1 2; do
for v in 256 128 64; do
  ADAPTSEG_X3R_FWD_MIN_CIN=$v timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abx.json 2>gpurun_out/abx.err || { tail -5 gpurun_out/abx.err; exit 4; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abx.json').read().strip().splitlines()[-1]); print('min_cin', sys.argv[1], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" "$v"
done
done
