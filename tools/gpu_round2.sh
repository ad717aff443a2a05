#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$tag.log 2>&1; local rc=$?; echo "bench $tag rc=$rc"; python -c "import json; d=json.loads(open('$O/bench_$tag.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['maximum_path']['ms_per_call'], d['losses'])" 2>/dev/null || tail -5 $O/bench_$tag.log; return $rc; }
run graph_bf16 || exit $?
run graph_f32 --precision 32-true || exit $?
run eager_bf16 --no-graph || exit $?
