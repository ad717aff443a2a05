#!/bin/bash
# glue in HIP (masks, duration loss, loss sum, time MLP): op tests, the whole suite, bench + step breakdown
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3c}; mkdir -p $O; cd $R
timeout -k 10 200 python -u -m pytest tests/test_step_glue_gpu.py -x -q --timeout 120 --timeout-method thread > $O/glue_tests.log 2>&1; rc=$?
tail -3 $O/glue_tests.log; [ $rc -ne 0 ] && { grep -B5 -A25 "Error\|assert" $O/glue_tests.log | head -80; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" $O/gpu_tests.log | head -80; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --steps 10 --warmup 3 > $O/prof_bench.json 2> $O/prof_err.log; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof_err.log; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step_breakdown.txt; head -45 $O/step_breakdown.txt
cd $R && timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cut -c1-250 $O/bench.json; exit $rc
