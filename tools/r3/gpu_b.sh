#!/bin/bash
# weight- vs activation-rounding split of the bf16 loss error; the new glue-op tests
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3b}; mkdir -p $O; cd $R
timeout -k 10 300 python tools/r3/precision_budget.py default > $O/precision_budget.jsonl 2> $O/precision_budget.err; rc=$?
echo "budget rc=$rc"; cat $O/precision_budget.jsonl | cut -c1-1500; [ $rc -ne 0 ] && { tail -20 $O/precision_budget.err; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_step_glue_gpu.py tests/test_headline_gpu.py tests/test_training_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --steps 10 --warmup 3 > $O/prof_bench.json 2> $O/prof_err.log; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof_err.log; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step_breakdown.txt; head -40 $O/step_breakdown.txt
