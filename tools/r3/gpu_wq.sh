#!/bin/bash
# same-box A/B: this session's code vs the first session's final (73910e3, copied into ab_old/, not committed)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wq}; mkdir -p $O
for rep in 1 2 3; do for tree in old new; do
  if [ $tree = old ]; then cd $R/ab_old; else cd $R; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$tree rep $rep', d['ms_per_step'], d['value'])"
done; done
