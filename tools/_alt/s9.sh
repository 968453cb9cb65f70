cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 800 bash tools/ab.sh "tests/test_gpu_xcdm.py" "python -u tools/time_any.py --mode MOL --L 4000 --B 10,32,115" xmh2a0 xmh2a6 > gpurun_out/r06_ab_xcdm_h2at.log 2>&1
