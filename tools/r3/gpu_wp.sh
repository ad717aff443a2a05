#!/bin/bash
# unrolled loss kernels + embedding backward on the side stream: tests, profile, bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wp}; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests/test_training_gpu.py tests/test_step_glue_gpu.py tests/test_encoder_ops_gpu.py tests/test_headline_gpu.py tests/test_model_gpu.py tests/test_dp_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -2 $O/step.txt; grep -E "loss_|embedding" $O/step.txt
cd $R
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('rep $rep', d['ms_per_step'])"
done
