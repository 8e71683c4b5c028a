#!/bin/bash
# Counters of every kernel of one bench step, in the step (kernel trace) and alone (--pmc passes,
# which serialise the dispatches): summarised by tools/step_pmc.py.  One counter set per run, no
# trace domains with --pmc; each pass under its own KILL limit.
#   bash tools/gpu_step_pmc.sh CFG   ->  gpurun_out/step_pmc_CFG/{trace,p1..p4}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${1:-c2}
OUT=$R/gpurun_out/step_pmc_$CFG
mkdir -p $OUT
cd /tmp
B="python3 $R/bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --no-roofline"
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || exit 3
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $SET -d $OUT/p$i -o run --output-format csv -- $B > $OUT/p$i.log 2>&1 || exit $((3 + i))
done
echo STEP_PMC_OK
