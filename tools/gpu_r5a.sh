#!/bin/bash
# Round 5, first GPU call: the bench-batch parity tests, per-shape conv tables (c2, c4), and the
# counters of the c2 step (time-dominant kernel: traffic + MFMA / VALU / stall split in the step
# and alone, tools/gpu_step_pmc.sh), plus conv_bench isolation passes of the 1x1 layer-3 convs.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5a
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest tests/test_fullres_gpu.py -v --timeout 600 --timeout-method thread \
  -k "bench_batch or B8" > $O/pytest_batch.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --reps 5 > $O/conv_shapes_c2.txt 2>&1 || exit 3
timeout -k 10 400 python -u tools/conv_bench.py --math f32x3 --reps 3 --model vgg --batch 8 > $O/conv_shapes_c4.txt 2>&1 || exit 4
bash tools/gpu_step_pmc.sh c2 || exit 5
bash tools/gpu_pmc.sh l3c3 l3.conv3 "--math f32x3" || exit 6
echo R5A_OK
