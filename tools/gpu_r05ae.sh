#!/bin/bash
# Round 5 A/B: many-row GRU2 epilogue operands hoisted above the barrier + the three partials'
# loads issued together; deepmind R·h row sums' loads issued together (in-tree) vs HEAD.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_xcdm.py tests/test_gpu_xcdm_raw.py tests/test_gpu_dx.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ae_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05ae_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --L 3000 --B 10,32,64,115 --paths xcdm 2>&1 | grep us/step || exit 1
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode RAW --L 3000 --B 1,115 --paths xcdm 2>&1 | grep us/step || exit 1
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 32 2>&1 | grep us/step || exit 1
done
