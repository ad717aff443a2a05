#!/bin/bash
# duration-predictor branch stream: tests + same-box A/B; then the 96-row tile sweep of the decoder GEMMs
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wi}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_dp_gpu.py tests/test_headline_gpu.py tests/test_model_gpu.py tests/test_dp_multirank_gpu.py tests/test_encoder_ops_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do for b in 1 0; do
  MTTS_BRANCH_STREAM=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('branch=$b rep $rep', d['ms_per_step'])"
done; done
SWEEP_GLDS=32-51 SWEEP_SPLITS=1 SWEEP_REG=1 SWEEP_MIN_ROWS=9600 timeout -k 10 700 python -u tools/r3/gemm_step_sweep.py > $O/sweep.jsonl 2> $O/sweep.err; rc=$?
tail -2 $O/sweep.err; wc -l $O/sweep.jsonl; exit $rc
