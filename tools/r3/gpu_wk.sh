#!/bin/bash
# first micro-batch of an accumulating step deferred: tests + the bench's extra configs (16x2 reference step)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wk}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_dp_multirank_gpu.py tests/test_dp_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-synth --no-graph-profile --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'])
print({k: v['ms_per_step'] for k, v in d['extra_configs'].items()})"
