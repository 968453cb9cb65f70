#!/bin/bash
# A/B of alternative builds of the library (tools/_alt/*.so) on the multi-row kernel
# (tools/ab_rows.py: oracle parity + device us/step at B = 115, 32, 10), the in-tree build first
# and last (box drift).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 200 python -u tools/ab_rows.py DUMMY=0 ${@:-115 32 10} 2>&1 | grep -E "B=|Error" || exit $?
done
