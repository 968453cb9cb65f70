#!/bin/bash
# Round 5 A/B: the XCD kernels' wave index through readfirstlane (uw: dense + sparse, uws: sparse only).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
( TIME_DM_LIB=$PWD/tools/_alt/uw.so timeout -k 10 300 python -u tools/parity_any.py --B 1,8 --L 400 --path xcd &&
  TIME_DM_LIB=$PWD/tools/_alt/uw.so timeout -k 10 300 python -u tools/parity_any.py --B 1,8 --L 400 --path xcd --rnn 896 --prune 0.95 ) > gpurun_out/r05o_par.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05o_par.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/uw.so tools/_alt/uws.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/uw.so tools/_alt/uws.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
done
