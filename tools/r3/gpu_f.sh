#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3f}; mkdir -p $O; cd $R
timeout -k 10 200 python -u -m pytest tests/test_step_glue_gpu.py -x -q --timeout 120 --timeout-method thread > $O/glue_tests.log 2>&1; rc=$?
tail -2 $O/glue_tests.log; [ $rc -ne 0 ] && { grep -B5 -A25 "Error\|assert " $O/glue_tests.log | head -60; exit $rc; }
timeout -k 10 200 python tools/r3/weight_sensitivity.py > $O/sensitivity.jsonl 2> $O/sensitivity.err; rc=$?
echo "sens rc=$rc"; [ $rc -ne 0 ] && { tail $O/sensitivity.err; exit $rc; }
python -c "
import json
for l in open('$O/sensitivity.jsonl'):
    d=json.loads(l); print(d['loss'], d['value'], 'pred', d['pred_rel_err_rms'])
    for r in d['ranked'][:25]: print('   ', r)"
MTTS_W_SPLIT=0 timeout -k 10 200 python tools/r3/glue_map.py $O/glue_map.txt > /dev/null 2> $O/glue.err; echo "glue rc=$?"; head -60 $O/glue_map.txt
cd /tmp; export TMPDIR=/tmp
MTTS_W_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -16 $O/step.txt; grep rows_gemm $O/step.txt
