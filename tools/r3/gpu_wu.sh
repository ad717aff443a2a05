#!/bin/bash
# encoder gradients side-flushed in chunks after the seam: same-box A/B of the chunk size
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wu}; mkdir -p $O; cd $R
for rep in 1 2 3; do for n in 0 24 32 40 48 64; do
  MTTS_ENC_SIDE_JOBS=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 30 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('enc_side_jobs=$n rep $rep', d['ms_per_step'])"
done; done
