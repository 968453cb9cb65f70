#!/bin/bash
# A/B of alternative builds of the library (tools/_alt/*.so) on the XCD-resident kernel, one
# process per build, the in-tree build first and last (box drift).  Timing: tools/diag_xcd.py.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/diag_xcd.py ${1:-20000} 2>&1 | grep -E "parity B=1 L=400|round|Error" || exit $?
done
