#!/bin/bash
# F32X3 wide multi-tap forwards on the term-image kernel with per-call images
# (ADAPTSEG_X3R_FWD_PERCALL; build the arm first: make -C adaptsegnet_amd/csrc BUILD=build_pc
# OUT=../lib/libadaptseg_pc.so EXTRA=-DADAPTSEG_X3R_FWD_PERCALL=1): parity, then c4 / c2 arms.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/libadaptseg_pc.so timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_x3_terms_gpu.py tests/test_model_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_percall.log 2>&1 || { tail -30 gpurun_out/pt_percall.log; exit 3; }
tail -1 gpurun_out/pt_percall.log
bash experiments/ab_grid.sh "libadaptseg.so:- libadaptseg_pc.so:-" 2 --config c4 --steps 6 --warmup 2 && \
bash experiments/ab_grid.sh "libadaptseg.so:- libadaptseg_pc.so:-" 2 --config c2 --steps 10 --warmup 3
