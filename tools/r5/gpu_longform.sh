#!/bin/bash
# round 5 long-form lines (config 5's single-GPU workload: B = 8, Tx 512, Ty 4096): max-length and bucketed
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5longform}; mkdir -p $O; cd $R
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --no-extra --no-cpu-baseline --no-synth > $O/longform_max.json 2> $O/lf1.err || { tail -5 $O/lf1.err; exit 1; }
python tools/r5/bench_summary.py $O/longform_max.json 2>/dev/null | head -3
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --bucketed 4 --no-extra --no-cpu-baseline --no-synth --no-graph-profile > $O/longform_bucketed.json 2> $O/lf2.err || { tail -5 $O/lf2.err; exit 1; }
python tools/r5/bench_summary.py $O/longform_bucketed.json 2>/dev/null | head -3
