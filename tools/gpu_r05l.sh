#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
GRU2_STAMPS=1 TIME_DM_LIB=$PWD/tools/_alt/xcdsg.so timeout -k 10 120 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/r05l_stamps.log 2>&1 || { tail -5 gpurun_out/r05l_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05l_stamps.log
