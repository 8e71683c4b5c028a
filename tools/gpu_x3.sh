export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "f32x3 or accuracy" > gpurun_out/pytest_x3a.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_x3a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/conv_bench.py --math f32 --reps 3 > gpurun_out/convb_f32.txt 2>&1 || exit 5
timeout -k 10 300 python -u tools/conv_bench.py --math f32x3 --reps 3 > gpurun_out/convb_x3.txt 2>&1 || exit 6
tail -4 gpurun_out/convb_f32.txt; tail -4 gpurun_out/convb_x3.txt
