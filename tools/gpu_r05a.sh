#!/bin/bash
# Round 5: drop-in generate() at BASELINE sizes vs the reference, xcdm 3-quad parity, then the bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate_baseline.py tests/test_gpu_xcdm.py tests/test_gpu_xcdm_raw.py \
  -v -k "baseline or 80" --timeout 200 --timeout-method thread > gpurun_out/r05a_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r05a_pt.log | head -30; tail -3 gpurun_out/r05a_pt.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u bench.py > gpurun_out/r05a_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r05a_bench.log | cut -c1-600
