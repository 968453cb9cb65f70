#!/bin/bash
# Round 4: frame-terms parity after the interp rewrite + kernel breakdown of the drop-in calls.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame_terms.py -q --timeout 200 --timeout-method thread \
  > gpurun_out/frames_pt.log 2>&1 || { tail -30 gpurun_out/frames_pt.log; exit 1; }
tail -2 gpurun_out/frames_pt.log
AB_ONLY=frames timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_many8 -o run --output-format csv \
  -- python3 tools/ab_frames.py 1 many8 b1 fold60s > gpurun_out/prof_many8.log 2>&1 || exit $?
grep -E "x RT" gpurun_out/prof_many8.log
f=$(find gpurun_out/prof_many8 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -8
