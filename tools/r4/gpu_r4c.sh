#!/bin/bash
# round 4: suite + bench (default, with extras) + same-box A/B of the split-weight picker + parity step profile +
# the forced-DP step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4c}; mkdir -p $O; cd $R
TAG=${TAG:-r4c} bash tools/r4/gpu_suite.sh || exit $?
for i in 1 2; do
  for F in 0 1; do
    MTTS_GEMM_WS_PICK=$F timeout -k 10 200 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_ws$F.$i.json 2>/dev/null || exit $?
    echo "ws_pick=$F run $i: $(python -c "import json; d=json.loads([l for l in open('$O/ab_ws$F.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'])")"
  done
done
TAG=${TAG:-r4c}/prof PREC=bf16-parity bash tools/r4/gpu_prof.sh > /dev/null || exit $?
head -3 $O/prof/step.txt; cat $O/prof/phases.txt
MTTS_FORCE_DP=1 TAG=${TAG:-r4c}/prof_dp PREC=bf16-parity bash tools/r4/gpu_prof.sh > /dev/null || exit $?
head -3 $O/prof_dp/step.txt; cat $O/prof_dp/phases.txt
