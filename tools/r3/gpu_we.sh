#!/bin/bash
# batched wgrads with the batched split plan: full GPU suite, then same-box A/B of plan knobs
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3we}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/gpu_tests.log | head -40; exit $rc; }
for rep in 1 2; do for cfg in "128 1536" "96 1536" "192 1536" "128 2304" "128 1024"; do set -- $cfg
  MTTS_WGRAD_BMINBLK=$1 MTTS_WGRAD_BROWS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('bminblk=$1 brows=$2 rep $rep', d['ms_per_step'])"
done; done
