cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_v3_pytest_gpu.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/r06_v3_pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_v3_smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/r06_v3_bench.json 2> gpurun_out/r06_v3_bench.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_v3_prof -o run --output-format csv -- python bench.py --pmc 0 --cpu-steps 0 > gpurun_out/r06_v3_prof.out 2>&1 || exit 4
