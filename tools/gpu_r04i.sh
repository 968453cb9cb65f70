#!/bin/bash
# Round 4: stamps of the deepmind (32 rows) and many-row (115 rows) kernels.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 180 python -u tools/stamps_dx.py 32 2000 > gpurun_out/stamps_dx.log 2>&1 || { tail -5 gpurun_out/stamps_dx.log; exit 1; }
timeout -k 10 180 python -u tools/stamps_xcdm.py 115 > gpurun_out/stamps_xcdm.log 2>&1 || { tail -5 gpurun_out/stamps_xcdm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_dx.log | head -25
