cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_philox.py tests/test_gpu_generate_sparse.py tests/test_gpu_melresnet.py -s > gpurun_out/r06_parity2.log 2>&1
echo rc=$? >> gpurun_out/r06_parity2.log
timeout -k 10 600 bash tools/ab.sh "" "python -u tools/time_dm.py 32" dxpw dxgb > gpurun_out/r06_ab_dx_pubwait.log 2>&1
echo rc=$? >> gpurun_out/r06_ab_dx_pubwait.log
timeout -k 10 600 bash tools/ab.sh "" "python -u tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd" xpw1 xpw2 > gpurun_out/r06_ab_xcd_pubwait.log 2>&1
echo rc=$? >> gpurun_out/r06_ab_xcd_pubwait.log
