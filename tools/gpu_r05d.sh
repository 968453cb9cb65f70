#!/bin/bash
# Round 5: deepmind per-wave gates (no end-of-step / post-coarse-sample barriers) and the sparse
# kernel's early h2 publish — parity, A/B vs the round-start build, stamps.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dx.py tests/test_gpu_deepmind.py tests/test_gpu_baseline_shapes.py \
  tests/test_gpu_xcds.py tests/test_gpu_many.py -q --timeout 300 --timeout-method thread > gpurun_out/r05d_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05d_pt.log; grep -E "^FAILED|^E  " gpurun_out/r05d_pt.log | head
[ $rc -eq 0 ] || exit $rc
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/a_head.so $base; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_dm.py 8 32 2>&1 | grep -E "us/step|Error" || exit $?
done
bash tools/ab_any.sh --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 8 --paths xcd > gpurun_out/r05d_ab_xcds.log 2>&1 || exit $?
cat gpurun_out/r05d_ab_xcds.log
timeout -k 10 120 python -u tools/stamps_dx.py 32 2000 > gpurun_out/r05d_stamps_dx.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/r05d_stamps_xcds.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r05d_stamps_dx.log | head -40; grep -v amdgpu.ids gpurun_out/r05d_stamps_xcds.log
