#!/bin/bash
# side-stream flush at the decoder/encoder seam: training tests, same-box A/B, profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wg}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_dp_gpu.py tests/test_headline_gpu.py tests/test_dp_multirank_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do for sf in 1 0; do
  MTTS_SIDE_FLUSH=$sf timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('side_flush=$sf rep $rep', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $T $O/trace.csv
python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -32 $O/step.txt
