#!/bin/bash
# GPU suite, two bench lines, and a kernel-trace profile of the graph step (no synthesise) -> gpurun_out/TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/b_$i.json 2>$O/b_$i.err || exit 1
  python -c "import json;r=json.load(open('$O/b_$i.json'));print('bench', r['value'], r['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --steps 10 --warmup 3 > $O/prof_bench.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; exit $rc
