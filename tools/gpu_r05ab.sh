#!/bin/bash
# Round 5: deepmind kernel phase stamps at 32 rows (current tree).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stamps_dx.py 32 > gpurun_out/r05ab_dx.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05ab_dx.log | head -70
