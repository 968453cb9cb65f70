#!/bin/bash
# Round 5 A/B: deepmind kernel — gate role on wave 3 + FMA-corrected label inputs (in-tree) vs
# gate wave 0 + label_x (g0) vs HEAD; labels bit-exact first.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dx.py tests/test_gpu_deepmind.py tests/test_gpu_baseline_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05r_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05r_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so tools/_alt/g0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so tools/_alt/g0.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 32 2>&1 | grep us/step || exit 1
done
