#!/bin/bash
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "pad or conv_fwd_dgrad_wgrad or large_grid" > gpurun_out/exp2_tests.log 2>&1; tail -2 gpurun_out/exp2_tests.log
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_model_gpu.py -k "discriminator or forward_backward or eval_bn" tests/test_vgg.py > gpurun_out/exp2_model.log 2>&1; tail -2 gpurun_out/exp2_model.log
bash tools/dbg/ab_libs.sh "libadaptseg.so libadaptseg_vp.so libadaptseg_vq.so" --math f32x3 || exit 3
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --filter conv1 > gpurun_out/exp2_thin.txt 2>&1
grep -E "stem|D.conv1" gpurun_out/exp2_thin.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/exp2_c2.json 2>/dev/null || exit 5
python -c "import json,sys; d=json.loads(open('gpurun_out/exp2_c2.json').read().strip().splitlines()[-1]); print('c2', round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', d['roofline']['frac'])"
