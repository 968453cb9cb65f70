#!/bin/bash
# Per-kernel A/B of library builds: rocprofv3 kernel-trace summaries of tools/time_any.py for the
# working tree's library and each tools/_alt/*.so (loop kernel and GEMMs timed separately).
#   bash tools/ab_prof.sh --mode MOL --L 3000 --B 115 --paths xcdm
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
base=wavernn_amd/_lib/libwavernn_amd.so
for lib in $base tools/_alt/*.so; do
  name=$(basename $lib .so)
  TIME_DM_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/abp_$name" -o k \
      --output-format csv -- python -u tools/time_any.py "$@" > gpurun_out/abp_$name.log 2>&1 || exit $?
  echo "== $lib"; grep "us/step" gpurun_out/abp_$name.log
  python - "$PWD/gpurun_out/abp_$name/k_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f"   {r['Name'][:70]:70s} calls {r['Calls']:>4s} total {float(r['TotalDurationNs'])/1e6:9.3f} ms avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
