#!/bin/bash
# A/B over settings "VAR1=a,VAR2=b ..." on one box (each arg = one comma-separated env assignment list)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $(echo $cfg | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/c_$i.json 2>$O/c_$i.err || exit 1
  python -c "import json;r=json.load(open('$O/c_$i.json'));print('$cfg', r['value'], r['ms_per_step'])"
done
