#!/bin/bash
# short-T attention kernels: attention tests, encoder tests, model tests; then the step breakdown
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3i}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_encoder_ops_gpu.py tests/test_model_gpu.py tests/test_headline_gpu.py -q --maxfail 6 --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error:|^E  " $O/tests.log | head -60; exit $rc; }
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -24 $O/step.txt; grep attn $O/step.txt
cd $R && timeout -k 10 200 python -u -m pytest tests/test_step_glue_gpu.py -q --timeout 100 --timeout-method thread > $O/glue_tests.log 2>&1; rc=$?
tail -2 $O/glue_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/glue_tests.log | head -30; exit $rc; }
timeout -k 10 200 python -u tools/r3/rows_bench.py > $O/rows_bench.txt 2>&1; echo "rows rc=$?"; cat $O/rows_bench.txt | tail -12
