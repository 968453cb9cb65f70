#!/bin/bash
# One GPU session: parity suite, PMC traffic passes, headline bench (reading the traffic just
# measured), rocprofv3 kernel-trace summary of the same bench command.
# Stops at the first step that ends abnormally (fault/abort/timeout), per the pool rules.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_gpu rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_$c" -o pmc --output-format csv -- \
      python "$R/bench.py" --steps 1 --warmup 0 --cpu-steps 0 --other-configs 1 --fold-batched 0 > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > /dev/null
export WRNN_PMC_PROFILE="$R/gpurun_out/pmc_traffic.json"
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- \
    python "$R/bench.py" --steps 2 --warmup 1 --cpu-steps 0 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
# the headline alone (no fold-batched line, no other configs): the XCD kernel's average dispatch
# in this summary is the headline launch that roofline.achieved is computed from
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_headline" -o bench --output-format csv -- \
    python "$R/bench.py" --steps 2 --warmup 1 --cpu-steps 0 --other-configs 0 --fold-batched 0 > gpurun_out/prof_headline.log 2>&1
rc=$?; echo "rocprof headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/prof_headline.log | cut -c1-200
