#!/bin/bash
# Deepmind XCD kernel: parity tests, then the in-tree library against each tools/_alt/*.so
# (in-tree first and last: box drift) at 8 and 32 rows.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dx.py tests/test_gpu_deepmind.py tests/test_gpu_baseline_shapes.py::test_config5_32_rows_bit_exact tests/test_gpu_many.py::test_deepmind_batch32_equals_single_rows -q --timeout 200 --timeout-method thread > gpurun_out/dx_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dx_pt.log; grep -E "^E |FAILED" gpurun_out/dx_pt.log | head -5
[ $rc -eq 0 ] || exit $rc
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 32 2>&1 | grep -E "us/step|Error" || exit $?
done
