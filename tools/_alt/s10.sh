cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 tools/mfma_poll > gpurun_out/r06_mfma_poll.log 2>&1
