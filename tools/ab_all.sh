#!/bin/bash
# A/B of alternative builds of the library (tools/_alt/*.so) on every loop kernel except the
# XCD one (tools/ab_xcd.sh): rows (B = 10, 115), deepmind (B = 32), split (B = 1).  One process
# per build and kernel, the in-tree build first and last (box drift).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 180 python -u tools/ab_rows.py DUMMY=0 10 115 2>&1 | grep -E "us/step|Error" || exit $?
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 32 2>&1 | grep -E "us|Error" || exit $?
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/ab_split.py DUMMY=0 30000 2>&1 | grep -E "us/step|Error" || exit $?
done
