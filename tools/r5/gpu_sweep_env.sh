#!/bin/bash
# step sweep of one environment switch over several values (VAR, VALS="a b c"), two alternating rounds on one box
# -> gpurun_out/$TAG/sweep.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5sweep}; mkdir -p $O; cd $R
X="--no-extra --no-synth --no-cpu-baseline --no-graph-profile --steps 40 --warmup 5 ${BENCH_ARGS}"
: > $O/sweep.txt
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py $X > $O/r.json 2> $O/r.err || { echo "$v failed"; tail -5 $O/r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/r.json').read().strip().splitlines()[-1]); print('$VAR=$v rep $rep', d['ms_per_step'], d.get('precision_check',{}).get('modes',{}).get('parity_policy',{}).get('loss_rel_err'))" >> $O/sweep.txt
  done
done
cat $O/sweep.txt
