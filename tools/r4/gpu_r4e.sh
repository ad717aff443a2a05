#!/bin/bash
# round 4: MAS shape sweep (with the MAS / long-form tests), training + headline tests (t drawn before the prefetch
# fork, early prefetch join), then the bench A/B of MTTS_PREFETCH_JOIN=mas / decoder -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4e}; mkdir -p $O; cd $R
TAG=${TAG:-r4e}/sweep bash tools/r4/gpu_mas_sweep.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_headline_gpu.py tests/test_model_gpu.py tests/test_dp_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|^E  " $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for J in mas decoder; do
    MTTS_PREFETCH_JOIN=$J timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_$J.$i.json 2>/dev/null || exit $?
    echo "join=$J run $i: $(python -c "import json; d=json.loads([l for l in open('$O/ab_$J.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'], d['precision_check']['modes']['parity_policy'], d['maximum_path']['fused_prior_maximum_path_ms'])")"
  done
done
