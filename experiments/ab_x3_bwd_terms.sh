#!/bin/bash
# F32X3 layer 3-4 conv2 backward on term images (engine.X3_BWD_TERMS, env ADAPTSEG_X3_BWD_TERMS):
# 0 = fp32 operands (round-3 program), 1 = weight gradient on y1's / dY2's terms, 2 = data gradient
# too.  Parity subset first, then c2 / c3 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_x3_terms_gpu.py tests/test_fullres_gpu.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_bwdterms.log 2>&1 || { tail -30 gpurun_out/pt_bwdterms.log; exit 3; }
  tail -1 gpurun_out/pt_bwdterms.log
fi
for CFG in ${CFGS:-c2 c3}; do
for rep in 1 2; do
for v in ${ARMS:-0 1 2}; do
  ADAPTSEG_X3_BWD_TERMS=$v timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abt.json 2>gpurun_out/abt.err || { tail -5 gpurun_out/abt.err; exit 4; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abt.json').read().strip().splitlines()[-1]); bk={k['selector']: round(k['frac'],3) for k in d['roofline']['by_kernel']}; print('bwdterms', sys.argv[1], sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', bk)" "$v" "$CFG"
done
done
done
