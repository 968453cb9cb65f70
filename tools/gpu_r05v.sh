#!/bin/bash
# Round 5 A/B: sparse kernel block-row sums reduce-scattered over the engine (in-tree) vs four row
# sums + select (rs0).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_xcds.py tests/test_gpu_frame_terms.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05v_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05v_pytest.log; [ $rc -eq 0 ] || exit $rc
TIME_DM_LIB=$PWD/tools/_alt/rs0.so timeout -k 10 300 python -u tools/parity_any.py --B 1,8 --L 400 --path xcd --rnn 896 --prune 0.95 2>&1 | grep -v amdgpu.ids || exit 1
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/rs0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/rs0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/rs0.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
done
