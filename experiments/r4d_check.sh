export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_bf16_gpu.py tests/test_bn_bf16_storage_gpu.py tests/test_fullres_gpu.py tests/test_model_gpu.py tests/test_x3_terms_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r4d.log 2>&1
tail -3 gpurun_out/pytest_r4d.log
rm -rf gpurun_out/mfma_f32x3
bash tools/gpu_mfma_util.sh f32x3 && python3 tools/mfma_util.py gpurun_out/mfma_f32x3 || exit 5
CFGS="c5" ROUNDS=2 bash experiments/ab_env.sh 'bf16g|ADAPTSEG_BF16_GRADS=1|' 'fp32g|ADAPTSEG_BF16_GRADS=0|' || exit 6
CFGS="c2" ROUNDS=2 bash experiments/ab_env.sh 'base||' 'overlap||--overlap' || exit 7
