#!/bin/bash
# wgrad with two bf16 row steps in flight: op tests under MTTS_WGRAD_DEPTH16=2, then an interleaved step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3s}; mkdir -p $O; cd $R
MTTS_WGRAD_DEPTH16=2 timeout -k 10 300 python -u -m pytest tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_model_gpu.py -q --maxfail 6 --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -40; exit $rc; }
for rep in 1 2; do
for cfg in "1 512" "2 512" "2 384" "2 256"; do
  set -- $cfg
  MTTS_WGRAD_DEPTH16=$1 MTTS_WGRAD_MINBLK16=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab_$1_$2_$rep.json 2> $O/ab_$1_$2_$rep.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab_$1_$2_$rep.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab_$1_$2_$rep.json')); print('depth16=$1 minblk16=$2 rep $rep', d['ms_per_step'])"
done
done
