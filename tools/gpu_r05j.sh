#!/bin/bash
# Round 5: the many-row kernel with 8 waves per workgroup (2 per SIMD, K window 64) vs 4 — timings.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,32,64,115 --paths xcdm > gpurun_out/r05j_ab.log 2>&1 || { cat gpurun_out/r05j_ab.log; exit 1; }
cat gpurun_out/r05j_ab.log
