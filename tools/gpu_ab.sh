#!/bin/bash
# A/B of schedule switches on one box: bench (no CPU baseline, no synth) per MTTS_GEMM_SCHED_OFF value
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
for v in "$@"; do
  MTTS_GEMM_SCHED_OFF=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/b_$v.json 2>$O/b_$v.err || exit 1
  python -c "import json;r=json.load(open('$O/b_$v.json'));print('$v', r['value'], r['ms_per_step'], r['roofline']['avg_launch_us'])"
done
