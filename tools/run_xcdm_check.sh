#!/bin/bash
# Many-row kernel: parity suites (MoL + RAW heads), then an A/B against tools/_alt/*.so.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xcdm.py tests/test_gpu_xcdm_raw.py -x -v --timeout 120 --timeout-method thread > gpurun_out/xcdm_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xcdm_pytest.log; grep -E "FAILED|^E " gpurun_out/xcdm_pytest.log | head -5
[ $rc -eq 0 ] || exit $rc
bash tools/ab_any.sh --mode MOL --L 3000 --B 1,10,32,64 --paths xcdm > gpurun_out/ab_xcdm.log 2>&1; cat gpurun_out/ab_xcdm.log
bash tools/ab_any.sh --mode RAW --L 3000 --B 1,10 --paths xcdm > gpurun_out/ab_xcdm_raw.log 2>&1; cat gpurun_out/ab_xcdm_raw.log
