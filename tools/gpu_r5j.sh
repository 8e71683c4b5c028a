#!/bin/bash
# Round 5: where the fused BN sums lose time — per-shape alone (tools/bnsum_bench.py) and the c2
# step's kernel times with and without them (kernel trace).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 python -u tools/bnsum_bench.py > $O/bnsum_bench.txt 2>&1 || { tail -20 $O/bnsum_bench.txt; exit 3; }
cat $O/bnsum_bench.txt
cd /tmp
for s in 1 0; do
  ADAPTSEG_BN_SUMS=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$s -o run --output-format csv -- \
    python3 $R/bench.py --config c2 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof_$s.log 2>&1 \
    || { tail -20 $O/prof_$s.log; exit 4; }
done
cd $R
for s in 1 0; do
  f=$(ls $O/prof_$s/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find $O/prof_$s -name '*kernel_stats.csv' | head -1)
  echo "== BN_SUMS=$s"; python tools/prof_summary.py "$f" 5 | head -16
done
echo R5J_OK
