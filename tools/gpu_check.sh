#!/bin/bash
# Focused GPU check: one test selection first (stops on a fault), then the full GPU suite, then
# bench lines.  bash tools/gpu_check.sh TAG "first pytest selection" "bench configs"
export TMPDIR=/tmp
TAG=${1:-chk}
FIRST=${2:-"tests/test_x3_terms_gpu.py"}
CFGS=${3:-"c2"}
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
# shellcheck disable=SC2086
timeout -k 10 600 python -u -m pytest $FIRST -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_first_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_first_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_run.sh $TAG "tests -m gpu" "$CFGS"
