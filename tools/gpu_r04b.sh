#!/bin/bash
# Round 4: xcdm fc3-local parity + A/B, the NCCL sharding tests, sparse/dense stamps.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_gpu_xcdm.py tests/test_gpu_baseline_shapes.py tests/test_gpu_sharding_nccl.py \
  -q --timeout 200 --timeout-method thread > gpurun_out/xcdm_pt2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/xcdm_pt2.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,32,64,115 --paths xcdm > gpurun_out/ab_fc3.log 2>&1 || exit $?
cat gpurun_out/ab_fc3.log
timeout -k 10 120 python -u tools/stamps_xcd.py 3000 1 > gpurun_out/stamps_sparse.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/stamps_xcd.py 3000 0 > gpurun_out/stamps_dense.log 2>&1 || exit $?
tail -15 gpurun_out/stamps_sparse.log
