#!/bin/bash
# Round 5: the c4 bench with VGG term images — with and without the live roofline instrumentation
# (the term-image programs ran 2-2.7x slower under bench.py's roofline than under
# tools/step_times.py in earlier runs).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5q
mkdir -p $O
for c in 512 256; do
  for rf in "--no-roofline" ""; do
    ADAPTSEG_VGG_TERMS=2 ADAPTSEG_VGG_TERMS_MIN_C=$c timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 \
      --no-cpu-baseline $rf > $O/b_${c}${rf}.json 2> $O/b_${c}${rf}.err || { tail -5 $O/b_${c}${rf}.err; exit 3; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('c4 t2 thr', sys.argv[2], sys.argv[3] or 'roofline', round(d['value'],3), round(d['ms_per_step'],2), r.get('kernel'), round(r.get('frac',0),3), [(k['selector'], round(k['frac'],3)) for k in r.get('by_kernel',[])])" $O/b_${c}${rf}.json $c "$rf"
  done
done
echo R5Q_OK
