#!/bin/bash
# Round 5: why DeeplabVGG on term images (VGG_TERMS 1 / 2) is slower: per-shape x3r times and a
# kernel trace of the c4 step under VGG_TERMS=2.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 400 python -u tools/conv_bench.py --math f32x3_presplit --reps 3 --model vgg --batch 8 > $O/conv_shapes_c4_presplit.txt 2>&1 || exit 3
cd /tmp
ADAPTSEG_VGG_TERMS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_t2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $GRAFT_REPO_ROOT/$O/t2.log 2>&1 || exit 4
echo R5E_OK
