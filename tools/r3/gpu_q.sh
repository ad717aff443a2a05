#!/bin/bash
# fused RoPE attention: attention / encoder / model / headline tests, step breakdown
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3q}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_encoder_ops_gpu.py tests/test_model_gpu.py tests/test_headline_gpu.py tests/test_step_glue_gpu.py -q --maxfail 6 --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -40; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -24 $O/step.txt; grep "attn\|rope" $O/step.txt
