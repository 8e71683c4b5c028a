#!/bin/bash
# Round 5: the 256-row term-image weight-gradient tile for Cout >= 1024 (DeeplabVGG fc6 / fc7)
# under F32X3 — experiment build (EXTRA=-DADAPTSEG_X3R_WGRAD_BM256_MIN_COUT=1024) vs in-tree.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5t
mkdir -p $O
ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/libadaptseg_bm256.so timeout -k 10 500 python -u -m pytest tests/test_vgg.py -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_vgg.log 2>&1 || { tail -20 $O/pytest_vgg.log; exit 3; }
tail -1 $O/pytest_vgg.log
for rep in 1 2 3; do
  for L in libadaptseg.so libadaptseg_bm256.so; do
    ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 \
      --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 4; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('ab c4', sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', [(k['selector'], round(k['frac'],3), round(k['kernel_ms_per_step'],1)) for k in r['by_kernel']], flush=True)" $O/b.json $L | tee -a $O/ab.txt
  done
done
echo R5T_OK
