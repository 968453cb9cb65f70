#!/bin/bash
# A/B of library builds on the GPU box: a parity run on the in-tree build, then one timing
# command per build, each in its own process (TIME_DM_LIB), the in-tree build first and the list
# repeated (box drift).  Builds: python tools/build_alt.py <name> <source.hip> -DFLAG=V → tools/_alt/<name>.so
#   tools/ab.sh "<pytest files>" "<timing commands (bash -c)>" <name>...
#   e.g. tools/ab.sh tests/test_gpu_dx.py "python -u tools/time_dm.py 8 32" ride0
#        tools/ab.sh tests/test_gpu_xcd.py "python -u tools/time_any.py --mode MOL --L 20000 --B 1,8 --paths xcd" packf2_0
# (round 5's one-off drivers, tools/gpu_r05*.sh in git history, were this with fixed arguments;
# stamps: tools/stamps_{xcd,xcdm,dx}.py, clocks: tools/clock_pmc.py)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; export TMPDIR=/tmp; mkdir -p gpurun_out
tests=$1; cmd=$2; shift 2
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest $tests -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
libs=(wavernn_amd/_lib/libwavernn_amd.so)
for n in "$@"; do libs+=("tools/_alt/$n.so"); done
for rep in 1 2 3; do
  for lib in "${libs[@]}"; do
    echo "== $lib"
    TIME_DM_LIB=$PWD/$lib timeout -k 10 300 bash -c "$cmd" 2>&1 | grep us/step || exit 1
  done
done
