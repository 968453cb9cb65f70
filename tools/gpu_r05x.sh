#!/bin/bash
# Round 5: phase stamps of the dense and sparse XCD kernels after the ISA fixes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
true
timeout -k 10 300 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/r05x_sparse.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05x_dense.log; grep -v amdgpu.ids gpurun_out/r05x_sparse.log
