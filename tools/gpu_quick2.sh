#!/bin/bash
# GPU: the given test files, then the default bench line (no CPU baseline)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python -m pytest "$@" -x -q -m gpu > $O/quick_tests.log 2>&1; rc=$?; tail -3 $O/quick_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_quick.json 2>&1; rc=$?; python -c "import json; d=json.loads(open('$O/bench_quick.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['losses'], d['roofline']['achieved'])" || tail -5 $O/bench_quick.json; exit $rc
