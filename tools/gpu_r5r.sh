#!/bin/bash
# Round 5: split-K targets after the staged weight gradient got faster — experiment builds
# (EXTRA=-DADAPTSEG_X3_WGRAD_TARGET=320/448, -DADAPTSEG_X3R_WGRAD_MIN_KSTEPS=16/64) against the
# in-tree build (384 / 32), arms alternating.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
O=gpurun_out/r5r
mkdir -p $O
run() {
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$2 timeout -k 10 300 python -u bench.py --config $1 --steps 10 --warmup 3 \
    --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 3; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ab', sys.argv[2], sys.argv[3], round(d['value'],3), 'img/s', round(d['ms_per_step'],2), 'ms', flush=True)" $O/b.json $1 $2 | tee -a $O/ab.txt
}
for rep in 1 2; do
  for L in libadaptseg.so libadaptseg_t320.so libadaptseg_t448.so libadaptseg_k16.so libadaptseg_k64.so; do run c2 $L; done
done
for L in libadaptseg.so libadaptseg_t320.so libadaptseg_t448.so libadaptseg_k16.so libadaptseg_k64.so; do run c3 $L; done
echo R5R_OK
