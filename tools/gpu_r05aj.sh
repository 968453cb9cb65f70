#!/bin/bash
# Round 5 A/B: deepmind h_c poll riding along row group B of R·h (loads at fine-half chunk 6, gate
# wave chunk 0; in-tree) vs the blocking poll after it (ride0), and two other issue chunks.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dx.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05aj_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05aj_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/ride0.so tools/_alt/at3g2.so tools/_alt/at6g4.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/ride0.so tools/_alt/at3g2.so tools/_alt/at6g4.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 32 2>&1 | grep us/step || exit 1
done
