#!/bin/bash
# Round 5: the register-staged F32X3 kernel with a compile-time stage (K loop unrolled by two,
# transposed-read offsets hoisted) and unpacked split arithmetic: parity, per-shape, and the c2 / c4
# step against the previous build (libadaptseg_base.so), arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_x3_terms_gpu.py tests/test_epilogue_paths_gpu.py tests/test_vgg.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --reps 5 > $O/conv_shapes_c2.txt 2>&1 || exit 4
B=$GRAFT_REPO_ROOT/adaptsegnet_amd/lib/libadaptseg_base.so
CFGS="c2 c4" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh "base|ADAPTSEG_LIBRARY=$B|" "new||" "newt1|ADAPTSEG_VGG_TERMS=1|" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5G_OK
