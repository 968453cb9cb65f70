#!/bin/bash
# Round 4: xcdm selective re-poll A/B, then the full checkpoint (tools/gpu_r04.sh).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,32,64,115 --paths xcdm > gpurun_out/ab_repoll.log 2>&1 || { cat gpurun_out/ab_repoll.log; exit 1; }
cat gpurun_out/ab_repoll.log
bash tools/gpu_r04.sh
