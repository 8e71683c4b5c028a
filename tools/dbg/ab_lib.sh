#!/bin/bash
# A/B one alternative build (adaptsegnet_amd/lib/libadaptseg_ab.so) against the default one:
# conv_bench on both (args: conv_bench arguments).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for L in adaptsegnet_amd/lib/libadaptseg.so adaptsegnet_amd/lib/libadaptseg_ab.so; do
  echo "== $L"
  timeout -k 10 200 python -u tools/dbg/with_lib.py $L tools/conv_bench.py "$@" || exit 4
done
