cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "split or dropin" -v --timeout 120 --timeout-method thread > gpurun_out/pytest_split.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_split.log; grep -E "FAIL|Error" gpurun_out/pytest_split.log | head -10; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/ab_split.py "$@" && timeout -k 10 200 python tools/stamps_split.py
