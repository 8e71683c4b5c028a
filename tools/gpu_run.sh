#!/bin/bash
# One GPU-box session: GPU tests (optionally a subset), then bench lines, each step under its
# own time limit; stops at the first step that faults / times out.
#   bash tools/gpu_run.sh TAG "pytest selection args" "bench configs"
# e.g. bash tools/gpu_run.sh r2a "tests -m gpu" "c2 c5"
export TMPDIR=/tmp
TAG=${1:-run}
SEL=${2:-"tests -m gpu"}
CFGS=${3:-c2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
if [ "$SEL" != "none" ]; then
  # shellcheck disable=SC2086
  timeout -k 10 1000 python -u -m pytest $SEL -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures: still bench
fi
[ "$CFGS" = "none" ] && exit 0
for cfg in $CFGS; do
  timeout -k 10 400 python -u bench.py --config "$cfg" --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_${cfg}_$TAG.json 2> gpurun_out/bench_${cfg}_$TAG.err || exit 4
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],1), 'ms', d.get('roofline',{}).get('frac'))" gpurun_out/bench_${cfg}_$TAG.json "$cfg"
done
