#!/bin/bash
# Round 5 A/B: dense kernel GRU2 dots reduce-scattered (in-tree) vs three e32dot (drs0).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_xcd.py tests/test_gpu_parity.py tests/test_gpu_generate_baseline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05w_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05w_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/parity_any.py --B 1,8 --L 400 --path xcd 2>&1 | grep -v amdgpu.ids || exit 1
for lib in wavernn_amd/_lib/libwavernn_amd.so tools/_alt/drs0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/drs0.so wavernn_amd/_lib/libwavernn_amd.so tools/_alt/drs0.so; do
  echo "== $lib"
  TIME_DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd 2>&1 | grep us/step || exit 1
done
