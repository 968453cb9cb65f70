cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_v4_pytest_gpu.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/r06_v4_pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_v4_smoke.log 2>&1 || exit 2
