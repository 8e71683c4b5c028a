#!/bin/bash
# Round 5: the bf16 LDS-DMA forward / data-gradient kernel for products with 64 <= N < 128 too
# (layer1's N = 64 products and D.conv2's stride-2 data gradient; half of the 128-wide column tile
# idle) instead of the register-staged bf16 kernel: parity, per-shape, c5 arms (libadaptseg_n64.so
# = -DADAPTSEG_G16_MIN_N=64 vs the default build).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5ad
mkdir -p $O
ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/libadaptseg_n64.so timeout -k 10 500 python -u -m pytest tests/test_bf16_gpu.py \
  tests/test_bn_bf16_storage_gpu.py "tests/test_fullres_gpu.py" -k "bf16 or c5" -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for L in libadaptseg.so libadaptseg_n64.so; do
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u tools/conv_bench.py --math bf16 --reps 5 \
    > $O/conv_bf16_$L.txt 2>&1 || { tail -5 $O/conv_bf16_$L.txt; exit 4; }
  tail -4 $O/conv_bf16_$L.txt
done
for rep in 1 2 3; do
  for L in libadaptseg.so libadaptseg_n64.so; do
    ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 \
      --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 5; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('ab c5', sys.argv[2], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', [(k['selector'], round(k['frac'],3)) for k in r['by_kernel']], flush=True)" $O/b.json $L | tee -a $O/ab.txt
  done
done
echo R5AD_OK
