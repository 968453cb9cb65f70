#!/bin/bash
# Round 4: MoL sampler with the value-only ordered argmax — parity, then A/B against the round-3 form.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xcd.py tests/test_gpu_xcds.py tests/test_gpu_xcdm.py tests/test_gpu_parity.py \
  -q --timeout 300 --timeout-method thread > gpurun_out/mol_pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/mol_pt.log; grep -E "^FAILED" gpurun_out/mol_pt.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/ab_any.sh --mode MOL --L 20000 --B 1,8 --paths xcd > gpurun_out/ab_mol_argmax.log 2>&1 || exit $?
bash tools/ab_any.sh --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 8 --paths xcd >> gpurun_out/ab_mol_argmax.log 2>&1 || exit $?
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,115 --paths xcdm >> gpurun_out/ab_mol_argmax.log 2>&1 || exit $?
cat gpurun_out/ab_mol_argmax.log
