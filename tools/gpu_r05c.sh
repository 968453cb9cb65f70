#!/bin/bash
# Round 5: sparse XCD kernel with four fc waves — parity, A/B vs HEAD~1 build, stamps; training test.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xcds.py tests/test_gpu_training_forward.py tests/test_gpu_many.py \
  -q --timeout 300 --timeout-method thread > gpurun_out/r05c_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05c_pt.log; grep -E "^FAILED|^E  " gpurun_out/r05c_pt.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/ab_any.sh --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 1,8 --paths xcd > gpurun_out/r05c_ab.log 2>&1 || exit $?
cat gpurun_out/r05c_ab.log
timeout -k 10 120 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/r05c_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r05c_stamps.log | tail -25
