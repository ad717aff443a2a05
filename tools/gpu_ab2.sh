#!/bin/bash
# A/B of an environment switch on one box: bash tools/gpu_ab2.sh VAR val1 val2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/b_$v.json 2>$O/b_$v.err || exit 1
  python -c "import json;r=json.load(open('$O/b_$v.json'));print('$VAR=$v', r['value'], r['ms_per_step'], r['roofline']['avg_launch_us'])"
done
