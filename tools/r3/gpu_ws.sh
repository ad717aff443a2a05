#!/bin/bash
# performance-only switches re-checked on the batched-gradient step (same box, interleaved)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3ws}; mkdir -p $O; cd $R
CFGS=("BASE=1" "MTTS_GEMM_SCHED_OFF=4" "MTTS_GEMM_SCHED_OFF=2" "MTTS_GEMM_SCHED_OFF=8" "MTTS_WGRAD_LIN=0" "MTTS_WGRAD_MINSTEPS=8" "MTTS_WGRAD_MINSTEPS=2" "MTTS_RESNET_DX_LINK=0" "MTTS_QKV_BIAS_ONE_CAT=0" "MTTS_ATTN_BWD_MERGED=0")
for rep in 1 2; do for c in "${CFGS[@]}"; do
  env $c timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { echo "$c failed"; tail -3 $O/ab.err; continue; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('$c rep $rep', d['ms_per_step'])"
done; done
