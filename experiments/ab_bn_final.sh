export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bn_bf16_storage_gpu.py tests/test_bf16_gpu.py tests/test_ops_gpu.py tests/test_x3_terms_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_bn.log 2>&1 || { tail -30 gpurun_out/pt_bn.log; exit 3; }
tail -1 gpurun_out/pt_bn.log
bash experiments/ab_grid.sh "libadaptseg_u1.so:- libadaptseg.so:-" 2 --config c5 --steps 10 --warmup 3 && bash experiments/ab_grid.sh "libadaptseg_u1.so:- libadaptseg.so:-" 2 --config c2 --steps 10 --warmup 3
