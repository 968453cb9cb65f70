#!/bin/bash
# Round 5: baseline-size drop-in parity (with the observed |Δ|), MelResNet small tiles parity + timing,
# training-backward determinism diagnosis.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate_baseline.py tests/test_gpu_melresnet.py tests/test_gpu_parity.py \
  -rA -q -k "baseline or melresnet or dropin" --timeout 200 --timeout-method thread > gpurun_out/r05b_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "max|bit-exact|passed|failed" gpurun_out/r05b_pt.log | head -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -u tools/time_melresnet.py > gpurun_out/r05b_mr.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r05b_mr.log
timeout -k 10 300 python -u tools/diag_train_det.py MOL 4 > gpurun_out/r05b_det_mol.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/diag_train_det.py RAW 4 > gpurun_out/r05b_det_raw.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r05b_det_mol.log gpurun_out/r05b_det_raw.log | cut -c1-150
