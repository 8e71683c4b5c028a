#!/bin/bash
# Round 5: F32X3 term-image weight gradient with a per-lane pixel walk (both tiles) and the
# 256-row tile's K loop unrolled over its two ring stages: parity, then c4 / c2 arms vs the previous build (base).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_ops_gpu.py tests/test_x3_terms_gpu.py tests/test_vgg.py "tests/test_fullres_gpu.py" -k "not bf16 and not c5" \
  -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for cfg in c4 c2; do
    for L in libadaptseg_base.so libadaptseg.so; do
      ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 \
        --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 5; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('ab', sys.argv[3], sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', [(k['selector'], round(k['frac'],3)) for k in r['by_kernel']], flush=True)" $O/b.json $L $cfg | tee -a $O/ab.txt
    done
  done
done
echo R5AA_OK
