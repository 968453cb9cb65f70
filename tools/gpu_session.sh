#!/bin/bash
# One GPU session: parity suite, the headline bench exactly as the driver runs it (its
# own live PMC passes included), rocprofv3 kernel-trace summaries of the bench and of the headline
# alone.  Stops at the first step that ends abnormally (fault / abort / timeout), per the pool rules.
#   tools/gpu_session.sh [pytest -k expression]   (SKIP_TESTS / SKIP_BENCH / SKIP_PMC / SKIP_PROF=1 skip a step)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
K="${1:-}"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${K:+-k "$K"} \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_gpu rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/bench.log > gpurun_out/bench.json
  cut -c1-400 gpurun_out/bench.json
fi
if [ -z "$SKIP_PMC" ]; then
  # the HBM traffic passes on their own (one counter per pass), summarised like bench.py's live ones
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_$c" -o pmc --output-format csv -- \
        python "$R/bench.py" --pmc-child > gpurun_out/pmc_$c.log 2>&1
    rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > /dev/null && echo "pmc summary ok"
fi
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- \
      python "$R/bench.py" --steps 2 --warmup 1 --cpu-steps 0 --pmc 0 > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_headline" -o bench --output-format csv -- \
      python "$R/bench.py" --steps 2 --warmup 1 --cpu-steps 0 --other-configs 0 --fold-batched 0 --pmc 0 \
      > gpurun_out/prof_headline.log 2>&1
  rc=$?; echo "rocprof headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/prof_headline.log | cut -c1-200
fi
