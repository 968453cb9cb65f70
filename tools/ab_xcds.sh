#!/bin/bash
# A/B of alternative builds of the library (tools/_alt/*.so) on the XCD-resident block-sparse
# kernel (rnn 896), one process per build, the in-tree build first and last.  Timing: tools/diag_xcds.py.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 180 python -u tools/diag_xcds.py ${1:-6000} 2>&1 | grep -E "parity B=1|xcd B=8|Error" || exit $?
done
