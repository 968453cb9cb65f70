#!/bin/bash
# Round 5 diag: many-row kernel with the carried state consumed before the loop (in-tree) vs HEAD,
# and a no-output-store diagnostic build (timing only).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_xcdm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ac_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05ac_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so tools/_alt/noout.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so tools/_alt/noout.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --L 3000 --B 10,32,115 --paths xcdm 2>&1 | grep us/step || exit 1
done
