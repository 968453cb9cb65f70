#!/bin/bash
# Round 5: many-row kernel phase stamps at 115 and 10 rows (current tree).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stamps_xcdm.py 115 > gpurun_out/r05af_b115.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stamps_xcdm.py 10 > gpurun_out/r05af_b10.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05af_b115.log | head -30; grep -v amdgpu.ids gpurun_out/r05af_b10.log | head -26
