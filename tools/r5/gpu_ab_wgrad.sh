#!/bin/bash
# step A/B of the batched weight-gradient split rule (MTTS_WGRAD_BROWS rows per split / MTTS_WGRAD_BMINBLK blocks
# per job), alternating on one box -> gpurun_out/$TAG/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5abwg}; mkdir -p $O; cd $R
A="--no-extra --no-synth --no-cpu-baseline --no-graph-profile --steps 40 --warmup 5"
: > $O/ab.txt
for rep in 1 2; do
  for v in "1536 128" "3072 128" "3072 64" "4608 64" "1024 128"; do
    set -- $v
    MTTS_WGRAD_BROWS=$1 MTTS_WGRAD_BMINBLK=$2 timeout -k 10 300 python bench.py $A > $O/r.json 2> $O/r.err || { echo "$v failed"; tail -5 $O/r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/r.json').read().strip().splitlines()[-1]); print('rows $1 minblk $2 rep $rep', d['ms_per_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
