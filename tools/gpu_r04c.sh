#!/bin/bash
# Round 4: frame-rate terms parity + A/B, xcdm fc3-local A/B.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_frame_terms.py tests/test_gpu_parity.py tests/test_gpu_many.py \
  -q --timeout 200 --timeout-method thread > gpurun_out/frames_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/frames_pt.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/ab_frames.py 2 > gpurun_out/ab_frames.log 2>&1 || exit $?
cat gpurun_out/ab_frames.log | grep -v amdgpu.ids
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,32,64,115 --paths xcdm > gpurun_out/ab_fc3.log 2>&1 || exit $?
cat gpurun_out/ab_fc3.log
