cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 bash tools/ab.sh "" "python -u tools/time_dm.py 8 32" dxnosplit dxsplit2 > gpurun_out/r06_ab_dx_gbsplit2.log 2>&1 || exit 1
TIME_DM_LIB=$PWD/tools/_alt/dxsplit2.so timeout -k 10 120 python -u tools/stamps_dx.py 32 > gpurun_out/r06_dx_stamps_gbsplit2.log 2>&1
