cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 bash tools/ab.sh "tests/test_gpu_dx.py tests/test_gpu_deepmind.py tests/test_gpu_philox.py" "python -u tools/time_dm.py 8 32" dxnosplit > gpurun_out/r06_ab_dx_gbsplit.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/stamps_dx.py 32 > gpurun_out/r06_dx_stamps_gbsplit.log 2>&1
