#!/bin/bash
# round 5 final snapshot: the whole GPU suite, smoke(), the default bench line, a rocprofv3 step profile
# -> gpurun_out/$TAG (copied to profiles/r05/final/)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5final}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r5/bench_summary.py $O/bench.json > $O/summary.txt; head -3 $O/summary.txt
TAG=${TAG:-r5final}/prof bash tools/r5/gpu_prof.sh > /dev/null || exit 1
head -3 $O/prof/step.txt
