#!/bin/bash
# Round 5: (1) the bf16 LDS-DMA forward / data gradient's bound — timing-only builds (dbg1: A rows
# from one L2 line, dbg2: B rows, dbg3: both, dbg4: no LDS-DMA); (2) the staged F32X3 kernel's
# incremental tap walk: parity, per-shape and step A/B against the previous build (base).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5o
mkdir -p $O
for L in libadaptseg_base.so libadaptseg_dbg1.so libadaptseg_dbg2.so libadaptseg_dbg3.so libadaptseg_dbg4.so; do
  echo "== $L"
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 200 python -u tools/conv_bench.py --math bf16 --reps 10 \
    --filter "l3.conv" > $O/$L.l3.txt 2>&1 || { tail -5 $O/$L.l3.txt; exit 3; }
  grep -E "^l3" $O/$L.l3.txt | grep -v " 2 " || true
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 200 python -u tools/conv_bench.py --math bf16 --reps 10 \
    --filter "l4.conv2" > $O/$L.l4.txt 2>&1 || { tail -5 $O/$L.l4.txt; exit 4; }
  grep -E "^l4" $O/$L.l4.txt | grep -v " 2 " || true
done
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_x3_terms_gpu.py tests/test_epilogue_paths_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/pytest_x3.log 2>&1 || { tail -30 $O/pytest_x3.log; exit 5; }
tail -1 $O/pytest_x3.log
for L in libadaptseg_base.so libadaptseg.so; do
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --reps 5 \
    > $O/conv_c2_$L.txt 2>&1 || { tail -5 $O/conv_c2_$L.txt; exit 6; }
  tail -4 $O/conv_c2_$L.txt
done
for rep in 1 2; do
  for cfg in c2 c4; do
    for L in libadaptseg_base.so libadaptseg.so; do
      ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 \
        --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 7; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ab', sys.argv[2], sys.argv[3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', flush=True)" $O/b.json $cfg $L | tee -a $O/ab.txt
    done
  done
done
echo R5O_OK
