#!/bin/bash
# Round 4: RAW sampler argmax (value-only max + single-lane ballot) — parity, then A/B.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xcdm_raw.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/raw_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/raw_pt.log; grep -E "^FAILED" gpurun_out/raw_pt.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/ab_any.sh --mode RAW --L 5000 --B 1,10,115 --paths xcdm > gpurun_out/ab_raw_argmax.log 2>&1 || exit $?
cat gpurun_out/ab_raw_argmax.log
