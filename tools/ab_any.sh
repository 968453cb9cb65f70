#!/bin/bash
# A/B of library builds (the working tree's, then each tools/_alt/*.so, then the working tree's
# again: box drift) on tools/time_any.py with the given arguments.
#   bash tools/ab_any.sh --mode MOL --B 1,10 --paths xcdm
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 180 python -u tools/time_any.py "$@" 2>&1 | grep -E "us/step|Error" || exit $?
done
