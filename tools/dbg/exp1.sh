#!/bin/bash
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
bash tools/dbg/ab_libs.sh "libadaptseg.so libadaptseg_va.so libadaptseg_vb.so libadaptseg_vc.so" --math f32x3 || exit 3
for v in base inline overlap; do
  if [ $v = inline ]; then S=tools/dbg/bench_inline_wgrad.py; X=""; elif [ $v = overlap ]; then S=bench.py; X="--overlap"; else S=bench.py; X=""; fi
  timeout -k 10 300 python -u $S --no-cpu-baseline --no-roofline --steps 10 --warmup 3 $X > gpurun_out/e1.json 2>/dev/null || exit 5
  python -c "import json,sys; d=json.loads(open('gpurun_out/e1.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" $v
done
