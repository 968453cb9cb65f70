#!/bin/bash
# A/B of the many-row kernel's local-GRU1 one-quad form (WRNN_XCDM_LOCAL=1) against the h1-hop form,
# plus stamps of the local form at 10 rows.
mkdir -p gpurun_out
for v in 0 1 0 1; do echo "== WRNN_XCDM_LOCAL=$v"; WRNN_XCDM_LOCAL=$v timeout -k 10 120 python tools/time_any.py --mode MOL --L 3000 --B 1,10,16 --paths xcdm 2>&1 | grep us/step || exit 1; done > gpurun_out/loc_time.log
cat gpurun_out/loc_time.log
WRNN_XCDM_LOCAL=1 timeout -k 10 120 python tools/stamps_xcdm.py 10 2000 > gpurun_out/st10loc.log 2>&1; head -48 gpurun_out/st10loc.log
