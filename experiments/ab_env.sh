#!/bin/bash
# Interleaved A/B of bench.py arms that differ by environment and / or bench arguments, one box.
#   CFGS="c2 c5" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 'name|ENV=1 ENV2=0|--bench-args' ...
# Prints one line per run (images/s, ms/step, the by_kernel live fractions).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for r in $(seq 1 "${ROUNDS:-2}"); do
  for cfg in ${CFGS:-c2}; do
    for arm in "$@"; do
      IFS='|' read -r name envs args <<< "$arm"
      out=gpurun_out/ab/${name}_${cfg}_${r}.json
      # shellcheck disable=SC2086
      env $envs timeout -k 10 300 python -u bench.py --config "$cfg" --steps "${STEPS:-10}" --warmup 3 \
        --no-cpu-baseline $args > "$out" 2> "${out%.json}.err" || { tail -5 "${out%.json}.err"; exit 3; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); bk={k['selector']: round(k['frac'],3) for k in d['roofline']['by_kernel']}; print('ab', sys.argv[2], sys.argv[3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', bk, flush=True)" "$out" "$cfg" "$name"
    done
  done
done
