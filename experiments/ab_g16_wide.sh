#!/bin/bash
# 256x256 bf16 LDS-DMA tiles: parity, per-shape (tools/conv_bench.py --math bf16) and c5 step,
# baseline lib (ADAPTSEG_G16_WIDE_MIN_TILES=0, ADAPTSEG_G16_WIDE_WGRAD=0), weight gradients only
# (libadaptseg_ww.so: MIN_TILES=0) and in-tree (both).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
A=${1:-libadaptseg_nw.so}
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_wide.log 2>&1 || { tail -30 gpurun_out/pt_wide.log; exit 3; }
tail -1 gpurun_out/pt_wide.log
ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$A timeout -k 10 300 python -u tools/conv_bench.py --math bf16 > gpurun_out/cs_nw.txt 2>&1 || exit 4
timeout -k 10 300 python -u tools/conv_bench.py --math bf16 > gpurun_out/cs_wide.txt 2>&1 || exit 5
bash experiments/ab_grid.sh "$A:- libadaptseg_ww.so:- libadaptseg.so:-" 2 --config c5 --steps 10 --warmup 3
