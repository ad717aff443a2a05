#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wx}; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; exit $rc
