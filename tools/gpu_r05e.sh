#!/bin/bash
# Round 5: the frames-rows entry (fold blocks) + the sharded folds on RCCL, sparse stamps.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame_rows.py tests/test_gpu_sharding_nccl.py tests/test_gpu_frame_terms.py \
  tests/test_gpu_generate_baseline.py -q --timeout 300 --timeout-method thread > gpurun_out/r05e_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05e_pt.log; grep -E "^FAILED|^E  " gpurun_out/r05e_pt.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/r05e_stamps_xcds.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r05e_stamps_xcds.log
