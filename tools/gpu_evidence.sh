#!/bin/bash
# Round evidence on one box: smoke(), the whole GPU suite (slowest tests listed), bench lines.
#   bash tools/gpu_evidence.sh TAG "bench configs"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
TAG=${1:-ev}; CFGS=${2:-c2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  --durations=40 > $O/pytest_gpu.log 2>&1
rc=$?
tail -45 $O/pytest_gpu.log | grep -E "passed|failed|s call|s setup" | head -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ "$CFGS" = "none" ] && exit 0
for cfg in $CFGS; do
  timeout -k 10 400 python -u bench.py --config "$cfg" --steps 10 --warmup 3 --no-cpu-baseline \
    > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit 4
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],1), 'ms', d['roofline']['kernel'], round(d['roofline']['frac'],3))" $O/bench_$cfg.json "$cfg"
done
