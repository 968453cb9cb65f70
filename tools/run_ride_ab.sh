#!/bin/bash
# A/B of the many-row kernel's ride-along issue chunk (tools/_alt/a_at*.so) at 32 / 64 / 115 rows
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_any.sh --mode MOL --L 3000 --B 10,64,115 --paths xcdm > gpurun_out/ab_ride.log 2>&1; rc=$?; cat gpurun_out/ab_ride.log; exit $rc
