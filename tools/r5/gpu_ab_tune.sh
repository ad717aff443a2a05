#!/bin/bash
# A/B of the GEMM schedule tuner (MTTS_GEMM_TUNE=0 vs default), alternating on one box -> gpurun_out/$TAG/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5abtune}; mkdir -p $O; cd $R
A="--no-extra --no-synth --no-cpu-baseline --no-graph-profile --steps 40 --warmup 5"
: > $O/ab.txt
for rep in 1 2; do
  for v in off on; do
    E=$([ $v = off ] && echo "MTTS_GEMM_TUNE=0" || echo "MTTS_GEMM_TUNE=1")
    env $E timeout -k 10 300 python bench.py $A > $O/$v$rep.json 2> $O/$v$rep.err || { echo "$v failed"; tail -5 $O/$v$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/$v$rep.json').read().strip().splitlines()[-1]); print('$v', $rep, d['ms_per_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
