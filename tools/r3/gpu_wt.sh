#!/bin/bash
# focused same-box A/B: GEMM schedule bit 8 off (register schedules instead of the lean 64x64 / q|k|v LDS-DMA ones)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wt}; mkdir -p $O; cd $R
CFGS=("BASE=1" "MTTS_GEMM_SCHED_OFF=8" "MTTS_GEMM_SCHED_OFF=8 MTTS_WGRAD_MINSTEPS=8")
for rep in 1 2 3 4; do for c in "${CFGS[@]}"; do
  env $c timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 30 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { echo "$c failed"; tail -3 $O/ab.err; continue; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$c rep $rep', d['ms_per_step'])"
done; done
