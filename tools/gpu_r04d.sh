#!/bin/bash
# Round 4: kernel breakdown of the 8-utterance drop-in with frame-rate terms.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
AB_ONLY=frames timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_many8 -o run -- python3 tools/ab_frames.py 1 many8 b1 > gpurun_out/prof_many8.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/prof_many8.log | tail -6
f=$(find gpurun_out/prof_many8 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -12
