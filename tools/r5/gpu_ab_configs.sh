#!/bin/bash
# step A/B over whole environment settings (CONFIGS: ';'-separated, each "VAR=v VAR2=w" or "default"), REPS rounds
# alternating on one box -> gpurun_out/$TAG/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5abcfg}; mkdir -p $O; cd $R
X="--no-extra --no-synth --no-cpu-baseline --no-graph-profile --steps 40 --warmup 5 ${BENCH_ARGS}"
: > $O/ab.txt
IFS=';' read -ra CS <<< "$CONFIGS"
for rep in $(seq 1 ${REPS:-3}); do
  for c in "${CS[@]}"; do
    e=$c; [ "$c" = "default" ] && e=""
    env $e timeout -k 10 300 python bench.py $X > $O/r.json 2> $O/r.err || { echo "$c failed"; tail -5 $O/r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/r.json').read().strip().splitlines()[-1]); print('$c', 'rep $rep', d['ms_per_step'], d.get('precision_check',{}).get('modes',{}).get('parity_policy',{}).get('loss_rel_err'))" >> $O/ab.txt
  done
done
cat $O/ab.txt
