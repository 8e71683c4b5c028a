#!/bin/bash
# round 4: c4 (DeeplabVGG) of the round-3 tree (_r3tree, commit 723ab3f, built here) vs this tree on
# one box, alternating — is round 4's lower c4 line the box or the code?
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out/ab
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab/c4_r4_$r.json 2> gpurun_out/ab/c4_r4_$r.err || exit 3
  (cd _r3tree && timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline) > gpurun_out/ab/c4_r3_$r.json 2> gpurun_out/ab/c4_r3_$r.err || exit 4
  for t in r4 r3; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ab c4', sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', round(d['roofline']['frac'],3))" gpurun_out/ab/c4_${t}_$r.json $t; done
done
