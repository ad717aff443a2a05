#!/bin/bash
# attention: 3 workgroups/CU decoder fwd, raw staging: tests, per-kernel trace at the decoder shape (bf16 storage), step breakdown
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3l}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_encoder_ops_gpu.py -q --maxfail 6 --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error:|^E  " $O/tests.log | head -60; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/attn600 -o run -- python3 $R/tools/attn_one.py 600 64 10 io16 > $O/attn600.log 2>&1; echo "attn rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -3 $O/step.txt; grep attn $O/step.txt
