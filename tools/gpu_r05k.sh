#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
TIME_DM_LIB=$PWD/tools/_alt/xcdm8.so timeout -k 10 300 python -u tools/parity_any.py --B 1,10,13,32,40,64 --L 300 > gpurun_out/r05k.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05k.log; [ $rc -eq 0 ] || exit $rc
TIME_DM_LIB=$PWD/tools/_alt/xcdm8.so timeout -k 10 300 python -u tools/parity_any.py --B 10 --L 12100 >> gpurun_out/r05k.log 2>&1
rc=$?; tail -2 gpurun_out/r05k.log; exit $rc
