#!/bin/bash
# Round 5: the F32X3_PRESPLIT program (every product on the term-image kernel) against the
# default on the current tree: per-shape isolation (conv_bench) and the c2 step, arms alternating;
# the float4 pool / bias-gradient kernels' parity and the c4 line with them.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "maxpool or conv" > $O/pytest_ops.log 2>&1 || { tail -30 $O/pytest_ops.log; exit 3; }
tail -2 $O/pytest_ops.log
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3_presplit --reps 5 > $O/conv_shapes_c2_presplit.txt 2>&1 || exit 4
CFGS="c2" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 'default||' 'presplit||--conv-math f32x3_presplit' > $O/ab.txt 2>&1 || exit 5
cat $O/ab.txt
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c4.json 2>$O/bench_c4.err || exit 6
tail -c 300 $O/bench_c4.json
echo R5B_OK
