#!/bin/bash
# conv_bench over several library builds: bash experiments/ab_libs.sh "libA.so libB.so ..." conv_bench args...
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 2
LIBS=$1; shift
for L in $LIBS; do
  echo "== $L"
  ADAPTSEG_LIBRARY=adaptsegnet_amd/lib/$L timeout -k 10 200 python -u tools/conv_bench.py "$@" | grep -E "^op|TOTAL" || exit 4
done
