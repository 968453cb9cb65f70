cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_v1_pytest_gpu.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/r06_v1_pytest_gpu.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r06_v1_bench.json 2> gpurun_out/r06_v1_bench.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_v1_prof -o run --output-format csv -- python bench.py --pmc 0 --cpu-steps 0 > gpurun_out/r06_v1_prof.out 2>&1 || exit 3
timeout -k 10 120 python -u tools/stamps_dx.py 32 > gpurun_out/r06_dx_stamps_b32.log 2>&1
timeout -k 10 120 python -u tools/stamps_dx.py 8 >> gpurun_out/r06_dx_stamps_b32.log 2>&1
timeout -k 10 600 bash tools/ab.sh "tests/test_gpu_dx.py tests/test_gpu_deepmind.py" "python -u tools/time_dm.py 8 32" dxold > gpurun_out/r06_ab_dx_pubbuf.log 2>&1
