#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xcds.py -q --timeout 200 --timeout-method thread > gpurun_out/r05m_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05m_pt.log; [ $rc -eq 0 ] || exit $rc
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/a_head.so wavernn_amd/_lib/libwavernn_amd.so; do
  echo "== $lib"; TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
done
GRU2_STAMPS=1 TIME_DM_LIB=$PWD/tools/_alt/xcdsg.so timeout -k 10 120 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/r05m_stamps.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05m_stamps.log
