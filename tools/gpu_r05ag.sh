#!/bin/bash
# Round 5 A/B: deepmind 448-wide hop rows padded to one 128-B line per workgroup (in-tree) vs unpadded (pad0).
#
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dx.py tests/test_gpu_deepmind.py tests/test_gpu_baseline_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ag_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05ag_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/pad0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/pad0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/pad0.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 16 24 32 2>&1 | grep us/step || exit 1
done
