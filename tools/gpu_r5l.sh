#!/bin/bash
# Round 5: ring depth of the bf16 LDS-DMA weight-gradient kernel (ADAPTSEG_G16_WGRAD_STAGES 3 vs
# deep): bf16 parity both ways, per-shape times, c5 arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5l
mkdir -p $O
for ns in 3 6; do
  ADAPTSEG_G16_WGRAD_STAGES=$ns timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 300 \
    --timeout-method thread > $O/pytest_bf16_$ns.log 2>&1 || { tail -30 $O/pytest_bf16_$ns.log; exit 3; }
  tail -1 $O/pytest_bf16_$ns.log
done
for ns in 3 6; do
  ADAPTSEG_G16_WGRAD_STAGES=$ns timeout -k 10 300 python -u tools/conv_bench.py --math bf16 --reps 5 \
    > $O/conv_bf16_$ns.txt 2>&1 || { tail -20 $O/conv_bf16_$ns.txt; exit 4; }
done
paste -d' ' <(awk '{printf "%-9s %2s %5s %5s %9s %9s\n",$1,$2,$8,$9,$11,$13}' $O/conv_bf16_3.txt) \
  <(awk '{printf "| %9s %9s\n",$11,$13}' $O/conv_bf16_6.txt) | grep -E "^conv| 2 " 
tail -4 $O/conv_bf16_3.txt; tail -4 $O/conv_bf16_6.txt
CFGS="c5" ROUNDS=3 STEPS=10 bash experiments/ab_env.sh 'ns3|ADAPTSEG_G16_WGRAD_STAGES=3|' \
  'ns6|ADAPTSEG_G16_WGRAD_STAGES=6|' > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5L_OK
