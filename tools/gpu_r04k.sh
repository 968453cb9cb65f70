#!/bin/bash
# Round 4: frame-entry edge tests; deepmind h_c hop stamps.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame_terms.py -q --timeout 200 --timeout-method thread > gpurun_out/frames_pt2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/frames_pt2.log; grep -E "^FAILED|^E " gpurun_out/frames_pt2.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 180 python -u tools/stamps_dx.py 32 2000 > gpurun_out/stamps_dx2.log 2>&1 || { tail -5 gpurun_out/stamps_dx2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_dx2.log | head -8
