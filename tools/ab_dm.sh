#!/bin/bash
# A/B of library builds (working tree, tools/_alt/*.so, working tree) on the deepmind kernels:
# device µs/step at the given row counts (tools/time_dm.py).   bash tools/ab_dm.sh 8 32
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py "$@" 2>&1 | grep -E "us|Error" || exit $?
done
