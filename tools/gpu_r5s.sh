#!/bin/bash
# Round 5: the VGG term-image program on by default (mode 2, >= 512 channels): its tests, the
# c4 arms against fp32 operands, and the timing-pool fix (bench roofline with the term-image data
# gradient as the roofline kernel, thr 256).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_vgg.py tests/test_fullres_gpu.py -x -q --timeout 600 --timeout-method thread \
  -k "vgg" > $O/pytest_vgg.log 2>&1 || { tail -30 $O/pytest_vgg.log; exit 3; }
tail -1 $O/pytest_vgg.log
ADAPTSEG_VGG_TERMS=2 ADAPTSEG_VGG_TERMS_MIN_C=256 timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 \
  --no-cpu-baseline > $O/b256.json 2> $O/b256.err || { tail -5 $O/b256.err; exit 4; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c4 t2 thr256 roofline', round(d['value'],3), round(d['ms_per_step'],2), r['kernel'], round(r['frac'],3))" $O/b256.json
CFGS="c4" ROUNDS=2 STEPS=10 bash experiments/ab_env.sh 'default||' 't0|ADAPTSEG_VGG_TERMS=0|' > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 5; }
cat $O/ab.txt
echo R5S_OK
