#!/bin/bash
# inline-flush threshold sweep with batched weight gradients (same box)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wc}; mkdir -p $O; cd $R
for rep in 1 2; do for n in 32 64 128 0; do
  MTTS_INLINE_REDUCE_JOBS=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab_$n_$rep.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab_$n_$rep.json')); print('inline=$n rep $rep', d['ms_per_step'])"
done; done
