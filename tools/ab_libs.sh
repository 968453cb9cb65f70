#!/bin/bash
# A/B of alternative builds of the library (tools/_alt/*.so) on the batch-1 split kernel, one
# process per build, the in-tree build first and last (box drift).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/ab_split.py DUMMY=0 ${1:-60000} || exit $?
done
