#!/bin/bash
# round 4 closing snapshot on HEAD (FF1 one plane in the parity policy): the whole GPU suite + smoke, the default
# bench line with extras, the parity-step rocprofv3 profile, the long-form lines -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4final4}; mkdir -p $O; cd $R
TAG=${TAG:-r4final4} SUITE=1 SMOKE=1 BENCH=1 bash tools/r4/gpu_suite.sh || exit $?
TAG=${TAG:-r4final4}/prof PREC=bf16-parity bash tools/r4/gpu_prof.sh || exit $?
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --no-extra --no-cpu-baseline --no-synth > $O/longform_max.json 2> $O/lf1.err || { tail -5 $O/lf1.err; exit 1; }
python tools/r4/bench_summary.py $O/longform_max.json 2>/dev/null | head -3
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --bucketed 4 --no-extra --no-cpu-baseline --no-synth --no-graph-profile > $O/longform_bucketed.json 2> $O/lf2.err || { tail -5 $O/lf2.err; exit 1; }
python tools/r4/bench_summary.py $O/longform_bucketed.json 2>/dev/null | head -3
echo final4-done
