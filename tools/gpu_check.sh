#!/bin/bash
# One GPU round: parity tests -> smoke -> bench -> rocprofv3 kernel trace.  Each GPU step has
# its own time limit; a crash/fault (rc > 1 for pytest) ends the round.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -s > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
# a device fault surfaces as ordinary test failures: stop before touching the GPU again
if grep -qiE "illegal memory access|memory access fault|hipErrorIllegalAddress" gpurun_out/pytest_gpu_$TAG.log; then exit 7; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || exit 4
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 5
cd $R && timeout -k 10 600 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_$TAG.log 2>&1 || exit 6
timeout -k 10 600 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.log 2>&1 || exit 8
# multi-rank rehearsal on one GPU (gloo): the N>1 code path of bench.py (broadcast, per-rank
# shards, gradient all-reduce, barrier + max-over-ranks timing)
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --batch 1 > gpurun_out/bench_dp2_gloo_$TAG.log 2>&1 || exit 9
timeout -k 10 600 python tools/bench_eval.py > gpurun_out/bench_eval_$TAG.log 2>&1 || exit 10
timeout -k 10 600 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.log 2>&1 || exit 11
timeout -k 10 300 python tools/bench_preprocess.py > gpurun_out/bench_preprocess_$TAG.log 2>&1 || exit 12
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --overlap > gpurun_out/bench_c2_overlap_$TAG.log 2>&1 || exit 13
bash tools/gpu_traffic.sh c2 || exit 14
timeout -k 10 600 python tools/bench_warper.py > gpurun_out/bench_warper_$TAG.log 2>&1 || exit 15
