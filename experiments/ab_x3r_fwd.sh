#!/bin/bash
# (historical: the ADAPTSEG_X3R_FWD / _MIN_CIN env switches it sets were removed from engine.py after
# the A/B; results in profiles/r3/x3r_forward_ab.txt)
# F32X3 conv2 forward (layers 3-4) on the term-image kernel with BN1 writing y1's terms
# (engine.x3_forward_terms; ADAPTSEG_X3R_FWD=0 turns it off): parity, then c2 / c3 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_fullres_gpu.py tests/test_x3_terms_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_x3rfwd.log 2>&1 || { tail -30 gpurun_out/pt_x3rfwd.log; exit 3; }
tail -1 gpurun_out/pt_x3rfwd.log
for CFG in c2 c3; do
for rep in 1 2; do
for v in 0 1; do
  ADAPTSEG_X3R_FWD=$v timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abx.json 2>gpurun_out/abx.err || { tail -5 gpurun_out/abx.err; exit 4; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abx.json').read().strip().splitlines()[-1]); bk={k['selector']: round(k['frac'],3) for k in d['roofline']['by_kernel']}; print('x3r_fwd', sys.argv[1], sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', bk)" "$v" "$CFG"
done
done
done
