#!/bin/bash
# two ranks sharing the one GPU: stdout must be exactly the one JSON line
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3ww}; mkdir -p $O; cd $R
MTTS_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/shared2.json 2> $O/shared2.err; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/shared2.err; exit $rc; }
wc -l $O/shared2.json
python -c "import json; d=json.load(open('$O/shared2.json')); print('shared-gpu 2 ranks', d['n_gpus'], d['ms_per_step'], d.get('dp'))"
