#!/bin/bash
# PMC counter passes (one --pmc set per run, no trace domains) over conv_bench on a filter.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-p}
FILT=${2:-l3.conv2}
EXTRA=${3:-}   # extra conv_bench.py arguments, e.g. "--math f32x3"
mkdir -p $R/gpurun_out/pmc_$TAG
cd /tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_$TAG/list.txt 2>&1 || true
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET -d $R/gpurun_out/pmc_$TAG/s$i -o run --output-format csv -- python3 $R/tools/conv_bench.py --filter $FILT --reps 3 $EXTRA > $R/gpurun_out/pmc_$TAG/s$i.log 2>&1
  rc=$?
  echo "set $i rc=$rc" >> $R/gpurun_out/pmc_$TAG/status.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
done
