#!/bin/bash
# GPU test suite + smoke + default bench line on one box -> gpurun_out/$TAG (round 4).
#   TAG=name SUITE=1 SMOKE=1 BENCH=1 BENCH_ARGS="..." bash tools/r4/gpu_suite.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4}; mkdir -p $O; cd $R
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 200 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1; rc=$?
  tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/gpu_tests.log | head -40; exit $rc; }
fi
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  tail -1 $O/smoke.log; [ $rc -ne 0 ] && { tail -20 $O/smoke.log; exit $rc; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 700 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err; rc=$?
  echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
  python tools/r4/bench_summary.py $O/bench.json
fi
