#!/bin/bash
# round 4: MAS / DP / training tests, the default bench line (extras: dp_forced_n1 with seam buckets), long-form lines
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4d}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_mas_gpu.py tests/test_dp_gpu.py tests/test_dp_multirank_gpu.py tests/test_training_gpu.py tests/test_longform_gpu.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .{0,200}" $O/tests.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python tools/r4/bench_summary.py $O/bench.json
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --no-extra --no-cpu-baseline --no-synth > $O/longform_max.json 2> $O/lf1.err || { tail -5 $O/lf1.err; exit 1; }
python tools/r4/bench_summary.py $O/longform_max.json
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --bucketed 4 --no-extra --no-cpu-baseline --no-synth --no-graph-profile > $O/longform_bucketed.json 2> $O/lf2.err || { tail -5 $O/lf2.err; exit 1; }
python tools/r4/bench_summary.py $O/longform_bucketed.json
