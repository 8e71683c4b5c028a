#!/bin/bash
# round 4: the fp32-MFMA / register-staged bf16 kernels back on the per-element epilogue (their
# batched read-back kinds removed: 82-97 instead of 184-217 VGPRs; libadaptseg.so) vs the head
# (libadaptseg_rbold.so), and the round-3 tree at c4: parity, then c4 / c2 / c5 on one box.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests/test_conv_coverage.py tests/test_ops_gpu.py tests/test_vgg.py tests/test_fullres_gpu.py \
  tests/test_bn_bf16_storage_gpu.py tests/test_mask_bits_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r4x.log 2>&1 || { tail -40 gpurun_out/pytest_r4x.log; exit 3; }
grep -E "passed|failed" gpurun_out/pytest_r4x.log | tail -1
L=adaptsegnet_amd/lib
CFGS="c4 c2 c5" ROUNDS=2 bash experiments/ab_env.sh 'new||' "old|ADAPTSEG_LIBRARY=$L/libadaptseg_rbold.so|" || exit 4
for r in 1 2; do
  (cd _r3tree && timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline) > gpurun_out/ab/c4_r3x_$r.json 2> gpurun_out/ab/c4_r3x_$r.err || exit 5
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ab c4 r3tree', round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms')" gpurun_out/ab/c4_r3x_$r.json
done
