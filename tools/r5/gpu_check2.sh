#!/bin/bash
# round 5: accumulation (stash + merged) and parity tests, then the bench line with extras
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5c2}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_headline_gpu.py tests/test_longform_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -s > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "grad norms|gradients vs|merged|FAILED|Error" $O/tests.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r5/bench_summary.py $O/bench.json > $O/summary.txt; cat $O/summary.txt
