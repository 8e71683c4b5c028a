#!/bin/bash
# Round 5 final tree: smoke() on the shipped library build, the multi-rank path rehearsed with
# 2 ranks on the one GPU (gloo; RCCL needs one GPU per rank) for c2 and c3, and the model /
# bf16 GPU tests on the same build.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for cfg in c2 c3; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-cpu-baseline --config $cfg \
    > $O/dp2_gloo_$cfg.json 2> $O/dp2_gloo_$cfg.err || { tail -20 $O/dp2_gloo_$cfg.err; exit 4; }
  tail -c 300 $O/dp2_gloo_$cfg.json; echo
done
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_bf16_gpu.py tests/test_dist_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 5; }
tail -1 $O/pytest.log
echo R5AC_OK
