#!/bin/bash
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --filter D.conv1 > gpurun_out/exp3_thin.txt 2>&1 && timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_vgg.py -k "discriminator or forward_backward or eval_bn or vgg" >> gpurun_out/exp3_thin.txt 2>&1 && timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --filter stem >> gpurun_out/exp3_thin.txt 2>&1 && timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 100 --timeout-method thread tests/test_ops_gpu.py -k pad >> gpurun_out/exp3_thin.txt 2>&1 || exit 2
grep -E "stem|D.conv1|passed|failed" gpurun_out/exp3_thin.txt
for rep in 1 2; do
for v in pad nopad; do
  if [ $v = nopad ]; then S=tools/dbg/bench_nopad.py; else S=bench.py; fi
  timeout -k 10 300 python -u $S --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > gpurun_out/e3.json 2>/dev/null || exit 5
  python -c "import json,sys; d=json.loads(open('gpurun_out/e3.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" $v
done
done
