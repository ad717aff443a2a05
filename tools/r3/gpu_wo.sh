#!/bin/bash
# decoder prefetch (weight packs + time path on the side stream beside the text encoder): tests, A/B, profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wo}; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests/test_training_gpu.py tests/test_dp_gpu.py tests/test_headline_gpu.py tests/test_model_gpu.py tests/test_dp_multirank_gpu.py tests/test_step_glue_gpu.py tests/test_longform_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do for pf in 1 0; do
  MTTS_PREFETCH=$pf timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('prefetch=$pf rep $rep', d['ms_per_step'], d['precision_check']['modes']['one_plane']['loss_rel_err'] if d.get('precision_check') else '')"
done; done
