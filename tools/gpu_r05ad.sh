#!/bin/bash
# Round 5 A/B: fc3 partial hand-off as tagged 8-byte LDS pairs polled by the consumer (one LDS round trip
# less) in the dense and sparse XCD kernels (in-tree) vs HEAD.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_xcd.py tests/test_gpu_xcds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ad_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05ad_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 1 --paths xcd 2>&1 | grep us/step || exit 1
done
