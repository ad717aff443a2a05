#!/bin/bash
# round 4: bf16x6 (three-plane) GEMM + encoder tests, the headline parity modes, then bench A/B of the parity
# policy's encoder forward (fp32fwd vs bf16x6)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4x6}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_weight_split_gpu.py tests/test_headline_gpu.py tests/test_pack_gpu.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .{0,200}|bf16-parity.*rel err" $O/tests.log | head -30; }
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
grep -E "rel err" $O/tests.log | head -20
for i in 1 2; do
  for E in fp32fwd bf16x6; do
    MTTS_PARITY_ENCODER=$E timeout -k 10 200 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_$E.$i.json 2>/dev/null || exit $?
    echo "encoder=$E run $i: $(python -c "import json; d=json.loads([l for l in open('$O/ab_$E.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'], d['precision_check']['modes']['parity_policy'])")"
  done
done
exit $rc
