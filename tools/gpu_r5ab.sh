#!/bin/bash
# Round 5 final tree: MFMA utilisation of the atrous convs under the bf16 conv math (c5) after the
# weight-gradient pixel walk (tools/gpu_mfma_util.sh bf16).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
bash tools/gpu_mfma_util.sh bf16 || exit 3
python3 tools/mfma_util.py gpurun_out/mfma_bf16 > gpurun_out/mfma_bf16_r5ab.txt || exit 4
cat gpurun_out/mfma_bf16_r5ab.txt
echo R5AB_OK
