#!/bin/bash
# capped grid for the side-flushed weight-gradient batch: tests + same-box A/B of the cap
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wl}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_decoder_ops_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do for cap in 0 96 160 256 384; do
  MTTS_SIDE_WGRAD_CAP=$cap timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('cap=$cap rep $rep', d['ms_per_step'])"
done; done
