#!/bin/bash
# Round 5: sparse XCD kernel per-step time vs rows and length (kernel trace).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; R=$PWD; mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/q" -o q --output-format csv -- \
  python3 -u $R/tools/time_any.py --mode MOL --rnn 896 --prune 0.95 --L 110275 --B 1,8,1,8 --paths xcd > $R/gpurun_out/q.log 2>&1 || exit 1
cd $R; grep us/step gpurun_out/q.log
f=$(ls gpurun_out/q/*kernel_trace.csv gpurun_out/q/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "xcds" in r["Kernel_Name"] or "Cijk" in r["Kernel_Name"]:
        print(r["Kernel_Name"][:50], r.get("Grid_Size_X", r.get("Grid_Size", "")), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, "ms")
PY
