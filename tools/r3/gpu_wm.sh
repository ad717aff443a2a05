#!/bin/bash
# long-form config 5 on one GPU with batched weight gradients: max-length batch and length-bucketed batches
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wm}; mkdir -p $O; cd $R
timeout -k 10 400 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --batch 8 --tx 512 --ty 4096 --steps 10 --warmup 3 > $O/longform_max.json 2> $O/lf1.err; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/lf1.err; exit $rc; }
python -c "import json; d=json.load(open('$O/longform_max.json')); print('max-length', d['ms_per_step'], d['value'])"
timeout -k 10 500 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --batch 8 --tx 512 --ty 4096 --bucketed 4 --steps 12 --warmup 8 > $O/longform_bucketed.json 2> $O/lf2.err; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/lf2.err; exit $rc; }
python -c "import json; d=json.load(open('$O/longform_bucketed.json')); print('bucketed', d['ms_per_step'], d['value'])"
# two ranks sharing the one GPU (gloo transport): the multi-GPU entry point end to end
MTTS_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/shared2.json 2> $O/shared2.err; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/shared2.err; exit $rc; }
python -c "import json; d=json.load(open('$O/shared2.json')); print('shared-gpu 2 ranks', d['n_gpus'], d['ms_per_step'], d.get('dp'))"
