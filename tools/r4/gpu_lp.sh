#!/bin/bash
# round 4: log-prior norm terms once per row / frame -- MAS + headline + long-form tests, the fused alignment
# timing and one bench line -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4lp}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_mas_gpu.py tests/test_longform_gpu.py tests/test_headline_gpu.py tests/test_model_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|^E  " $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/prior_mas_bench.py --configs 32x120x600,8x512x4096,8x1024x4096 --iters 30 > $O/prior.jsonl 2>/dev/null || exit $?
cat $O/prior.jsonl
timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/bench.json 2>/dev/null || exit $?
python tools/r4/bench_summary.py $O/bench.json | head -2
