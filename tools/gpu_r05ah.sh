#!/bin/bash
# Round 5: effective clock (GRBM_GUI_ACTIVE) of the deepmind and many-row kernels.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; R=$PWD; mkdir -p gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d "$R/gpurun_out/clkd" -o pmc --output-format csv -- \
  python3 -u $R/tools/time_dm.py 8 32 > $R/gpurun_out/clkd.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d "$R/gpurun_out/clkm" -o pmc --output-format csv -- \
  python3 -u $R/tools/time_any.py --mode MOL --L 3000 --B 10,115 --paths xcdm >> $R/gpurun_out/clkd.log 2>&1 || exit 1
cd $R; grep us/step gpurun_out/clkd.log
f=$(ls gpurun_out/clkd/*counter_collection.csv gpurun_out/clkd/*/*counter_collection.csv 2>/dev/null | head -1); python3 tools/clock_pmc.py $f deepmind_xcd
f=$(ls gpurun_out/clkm/*counter_collection.csv gpurun_out/clkm/*/*counter_collection.csv 2>/dev/null | head -1); python3 tools/clock_pmc.py $f xcdm
