cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deepmind.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_rows.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_rows.log; grep -E "FAIL|Error" gpurun_out/pytest_rows.log | head -10; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/stamps_rows.py "$@"
