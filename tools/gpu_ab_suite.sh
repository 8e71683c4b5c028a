#!/bin/bash
# Parity tests, per-shape conv times under two settings of one environment switch, and
# interleaved step A/B arms — one GPU call.
#   TESTS="tests/a.py ..." SHAPES="--math f32x3" SWITCH=ADAPTSEG_X3H VALUES="0 7" CFGS="c2" \
#     bash tools/gpu_ab_suite.sh TAG 'arm|ENV=..|args' ...
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
TAG=${1:-ab}; shift
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TESTS" ]; then
  # shellcheck disable=SC2086
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
  tail -1 $O/pytest.log
fi
if [ -n "$SWITCH" ]; then
  for v in $VALUES; do
    # shellcheck disable=SC2086
    env $SWITCH=$v timeout -k 10 300 python -u tools/conv_bench.py $SHAPES > $O/shapes_$v.txt 2>&1 || { tail -20 $O/shapes_$v.txt; exit 4; }
    grep -E "^op|TOTAL" $O/shapes_$v.txt
  done
fi
[ $# -eq 0 ] && exit 0
CFGS="${CFGS:-c2}" ROUNDS=${ROUNDS:-2} STEPS=10 bash experiments/ab_env.sh "$@" | tee $O/ab.txt || exit 5
