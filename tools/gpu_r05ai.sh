#!/bin/bash
# Round 5 A/B: dense XCD kernel hop F2 as packed floats with an "empty" pattern (one 128-B line per
# producer and slot, 4 sampler loads per lane) in-tree vs {value, tag} granules (packf2_0).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_xcd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ai_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05ai_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/packf2_0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/packf2_0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/packf2_0.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
done
