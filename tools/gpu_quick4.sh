#!/bin/bash
# all GPU tests + bench + kernel-trace profile -> gpurun_out/$1/
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-q4}; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/bench.json 2>$O/bench.err || exit 1
python -c "import json;r=json.load(open('$O/bench.json'));print(r['value'], r['ms_per_step'])"
bash tools/gpu_prof_bench.sh ${1:-q4}
