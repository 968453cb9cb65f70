#!/bin/bash
# Round 5: effective clock (GRBM_GUI_ACTIVE) of the XCD kernels at 1 row and 8 rows.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; R=$PWD; mkdir -p gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d "$R/gpurun_out/clk" -o pmc --output-format csv -- \
  python3 -u $R/tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd > $R/gpurun_out/clk.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d "$R/gpurun_out/clks" -o pmc --output-format csv -- \
  python3 -u $R/tools/time_any.py --mode MOL --rnn 896 --prune 0.95 --L 5000 --B 1,8 --paths xcd >> $R/gpurun_out/clk.log 2>&1 || exit 1
cd $R; grep us/step gpurun_out/clk.log
f=$(ls gpurun_out/clk/*counter_collection.csv gpurun_out/clk/*/*counter_collection.csv 2>/dev/null | head -1); python3 tools/clock_pmc.py $f xcd
f=$(ls gpurun_out/clks/*counter_collection.csv gpurun_out/clks/*/*counter_collection.csv 2>/dev/null | head -1); python3 tools/clock_pmc.py $f xcd
