#!/bin/bash
# Round 5 A/B: deepmind gates: all LDS operands issued at once, carried h consumed before the loop; sampler log q read before the poll (in-tree) vs HEAD.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dx.py tests/test_gpu_deepmind.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05z_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05z_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 32 2>&1 | grep us/step || exit 1
done
