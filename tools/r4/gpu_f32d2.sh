#!/bin/bash
# round 4: exact-fp32 register GEMMs with two K steps in flight (configs 18 / 11) -- bitwise test, parity /
# 32-true tests, then bench A/B of MTTS_GEMM_F32_DEPTH2 at bf16-parity and 32-true -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4f32}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_weight_split_gpu.py tests/test_headline_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|^E  " $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for D in 0 1; do
    MTTS_GEMM_F32_DEPTH2=$D timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_p$D.$i.json 2>/dev/null || exit $?
    MTTS_GEMM_F32_DEPTH2=$D timeout -k 10 300 python bench.py --precision 32-true --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 20 > $O/ab_t$D.$i.json 2>/dev/null || exit $?
    echo "depth2=$D run $i: parity $(python -c "import json; d=json.loads([l for l in open('$O/ab_p$D.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'], d['precision_check']['modes']['parity_policy'])") 32-true $(python -c "import json; d=json.loads([l for l in open('$O/ab_t$D.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'])")"
  done
done
