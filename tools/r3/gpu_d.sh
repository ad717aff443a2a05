#!/bin/bash
# split weight planes (bf16-mixed parity) + MFMA time MLP: op tests, headline parity, budget, same-box A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3d}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_weight_split_gpu.py tests/test_step_glue_gpu.py tests/test_decoder_ops_gpu.py tests/test_headline_gpu.py -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "rel err|agreement" $O/tests.log | head; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert " $O/tests.log | head -60; exit $rc; }
timeout -k 10 300 python tools/r3/precision_budget.py default > $O/precision_budget.jsonl 2> $O/precision_budget.err; rc=$?
echo "budget rc=$rc"; cut -c1-900 $O/precision_budget.jsonl; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do MTTS_W_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth > $O/bench_ws$v.json 2>> $O/bench.err || exit 1; python -c "import json;d=json.load(open('$O/bench_ws$v.json'));print('W_SPLIT=$v', d['ms_per_step'], d['precision_check']['bf16_loss_rel_err'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --steps 10 --warmup 3 > $O/prof_bench.json 2> $O/prof_err.log; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof_err.log; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step_breakdown.txt; head -40 $O/step_breakdown.txt
