cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab.sh "" "python -u tools/time_dm.py 8 32" dxpadl dxpade > gpurun_out/r06_ab_dx_padlate.log 2>&1
TIME_DM_LIB=$PWD/tools/_alt/dxpadl.so timeout -k 10 120 python -u tools/stamps_dx.py 32 > gpurun_out/r06_dx_stamps_padlate.log 2>&1
TIME_DM_LIB=$PWD/tools/_alt/dxpade.so timeout -k 10 120 python -u tools/stamps_dx.py 32 > gpurun_out/r06_dx_stamps_padearly.log 2>&1
