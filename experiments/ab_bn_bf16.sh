#!/bin/bash
# bf16-storage BN passes: parity, isolated (tools/bn_bench.py --bf16) and c5 step, arms alternating.
#   bash experiments/ab_bn_bf16.sh "A.so B.so ..."   (first arm = baseline)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
ARMS=${1:-"libadaptseg_u1.so libadaptseg.so"}
timeout -k 10 300 python -u -m pytest tests/test_bn_bf16_storage_gpu.py tests/test_bf16_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_bnbf16.log 2>&1 || { tail -30 gpurun_out/pt_bnbf16.log; exit 3; }
tail -1 gpurun_out/pt_bnbf16.log
for A in $ARMS; do
  echo "== isolated, $A"; ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$A timeout -k 10 200 python -u tools/bn_bench.py --bf16 2>&1 | grep -v amdgpu.ids || exit 4
done
L=""; for A in $ARMS; do L="$L $A:-"; done
bash experiments/ab_grid.sh "$L" 2 --config c5 --steps 10 --warmup 3
