#!/bin/bash
# Interleaved A/B of bench.py variants on the GPU box (methodology: alternate the variants in
# rounds inside ONE call, so clock / device drift hits every arm alike).
#
#   bash tools/ab.sh [-c "c2 c3"] [-r ROUNDS] [-s STEPS] NAME=ARGS [NAME=ARGS ...]
#
# ARGS are extra bench.py arguments (quote them), e.g.
#   bash tools/ab.sh -c "c2 c5" -r 2 base= overlap=--overlap
# Every run's JSON line goes to gpurun_out/ab/<name>_<config>_<round>.json and a table of
# images/s per arm is printed at the end.
set -o pipefail
CFGS="c2"; ROUNDS=2; STEPS=5
while getopts "c:r:s:" o; do
  case $o in c) CFGS=$OPTARG ;; r) ROUNDS=$OPTARG ;; s) STEPS=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
[ $# -ge 1 ] || { echo "usage: $0 [-c cfgs] [-r rounds] [-s steps] NAME=ARGS ..." >&2; exit 2; }
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  for cfg in $CFGS; do
    for arm in "$@"; do
      name=${arm%%=*}; args=${arm#*=}
      out=gpurun_out/ab/${name}_${cfg}_${r}.json
      # shellcheck disable=SC2086
      timeout -k 10 300 python -u bench.py --config "$cfg" --steps "$STEPS" --warmup 2 \
        --no-cpu-baseline $args > "$out" 2> "${out%.json}.err" || exit 3
      echo "round $r $cfg $name: $(python -c "import json,sys; print(round(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value'], 3))" "$out")"
    done
  done
done
