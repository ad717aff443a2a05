#!/bin/bash
# batched split plan re-checked with the chunked encoder flushes (same box, interleaved)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wy}; mkdir -p $O; cd $R
for rep in 1 2 3; do for cfg in "128 1536" "256 1536" "64 1536" "128 768"; do set -- $cfg
  MTTS_WGRAD_BMINBLK=$1 MTTS_WGRAD_BROWS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 30 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('bminblk=$1 brows=$2 rep $rep', d['ms_per_step'])"
done; done
