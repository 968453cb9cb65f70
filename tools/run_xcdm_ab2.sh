#!/bin/bash
# Many-row kernel: parity suites (MoL + RAW), A/B against tools/_alt/*.so at 32 / 64 / 115 rows,
# stamps at 115 rows.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xcdm.py tests/test_gpu_xcdm_raw.py -x -v --timeout 120 --timeout-method thread > gpurun_out/xcdm_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xcdm_pytest.log; grep -E "FAILED|^E " gpurun_out/xcdm_pytest.log | head -5
[ $rc -eq 0 ] || exit $rc
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,32,64,115 --paths xcdm > gpurun_out/ab_xcdm.log 2>&1; rc=$?; cat gpurun_out/ab_xcdm.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_any.sh --mode RAW --L 3000 --B 115 --paths xcdm > gpurun_out/ab_xcdm_raw.log 2>&1; rc=$?; cat gpurun_out/ab_xcdm_raw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/stamps_xcdm.py 115 2000 > gpurun_out/stamps_b115.log 2>&1; rc=$?; head -12 gpurun_out/stamps_b115.log; exit $rc
