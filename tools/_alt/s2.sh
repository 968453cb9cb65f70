cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_philox.py -s > gpurun_out/r06_philox_pytest.log 2>&1
echo rc=$? >> gpurun_out/r06_philox_pytest.log
