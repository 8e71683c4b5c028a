#!/bin/bash
# igemm_x3h_kernel: parity (tests/test_x3h_gpu.py), per-shape conv times with it off / on
# (tools/conv_bench.py under ADAPTSEG_X3H), and interleaved step A/B arms (experiments/ab_env.sh).
#   bash tools/gpu_x3h.sh TAG "cfgs" "arm ..."     (arm: 'name|ENV=..|bench args')
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
TAG=${1:-x3h}; CFGS=${2:-c2}; shift 2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_x3h_gpu.py tests/test_x3_terms_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for m in ${X3H_MODES:-0 7}; do
  ADAPTSEG_X3H=$m timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 > $O/conv_shapes_x3h$m.txt 2>&1 || { tail -20 $O/conv_shapes_x3h$m.txt; exit 4; }
  grep -E "^op|TOTAL" $O/conv_shapes_x3h$m.txt
done
[ $# -eq 0 ] && exit 0
CFGS="$CFGS" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh "$@" | tee $O/ab.txt || exit 5
