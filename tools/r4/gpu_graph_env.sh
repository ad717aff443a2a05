#!/bin/bash
# round 4: does the graph launch path cause the ~140 us of idle at the start of every replayed step (host-side
# packet submission)?  Bench A/B of the HIP runtime's graph submission knobs -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4g}; mkdir -p $O; cd $R
one() {  # $1 label, env set by caller
  timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_$1.json 2>/dev/null || return 1
  echo "$1: $(python -c "import json; d=json.loads([l for l in open('$O/ab_$1.json') if l.startswith('{')][-1]); print(d['ms_per_step'])")"
}
for i in 1 2; do
  one default.$i || exit 1
  DEBUG_HIP_GRAPH_BATCH_SIZE=4 one bs4.$i || exit 1
  DEBUG_HIP_GRAPH_BATCH_SIZE=16 one bs16.$i || exit 1
  DEBUG_HIP_GRAPH_BATCH_SIZE=64 one bs64.$i || exit 1
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 one nocap.$i || exit 1
done
