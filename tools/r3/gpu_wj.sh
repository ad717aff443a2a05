#!/bin/bash
# side-stream flushes of queued weight gradients in chunks during the backward (MTTS_SIDE_REDUCE) vs the seam flush
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wj}; mkdir -p $O; cd $R
for rep in 1 2; do for cfg in "0 24" "1 24" "1 48" "1 96"; do set -- $cfg
  MTTS_SIDE_REDUCE=$1 MTTS_SIDE_REDUCE_JOBS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('side_reduce=$1 jobs=$2 rep $rep', d['ms_per_step'])"
done; done
