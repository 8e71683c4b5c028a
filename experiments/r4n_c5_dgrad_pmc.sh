#!/bin/bash
# round 4: why the c5 bf16 1x1 data gradient (selector 194,
# igemm_bf16g_kernel<1,128,256,32>) runs 2-2.5x slower in the step than alone.  rocprofv3
# serialises dispatches while it collects counters, so the --pmc passes over the c5 step give each
# launch ALONE at its in-step shape; the kernel-trace pass gives the same launches concurrent
# with the weight-gradient stream.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c5pmc
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/trace.log 2>&1 || exit 3
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/p1.log 2>&1 || exit 4
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/p2.log 2>&1 || exit 5
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/p3 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/p3.log 2>&1 || exit 6
echo done
