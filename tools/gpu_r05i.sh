#!/bin/bash
# Round 5: deepmind single-launch timing + full GPU suite + bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/a_head.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 32 2>&1 | grep -E "us/step|Error" || exit $?
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05i_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05i_pt.log; grep -E "^FAILED" gpurun_out/r05i_pt.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u bench.py > gpurun_out/r05i_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r05i_bench.log | cut -c1-300
