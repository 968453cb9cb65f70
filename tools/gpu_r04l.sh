#!/bin/bash
# Round 4: fused MelResNet kernel — parity (kernel vs module, drop-in fixtures), then A/B.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_melresnet.py tests/test_gpu_parity.py tests/test_gpu_frame_terms.py tests/test_gpu_many.py \
  -q --timeout 300 --timeout-method thread > gpurun_out/mr_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/mr_pt.log; grep -E "^FAILED|^E  " gpurun_out/mr_pt.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_frames.py 2 b1 many8 fold60s > gpurun_out/ab_mr.log 2>&1 || exit $?
grep -E "x RT" gpurun_out/ab_mr.log
