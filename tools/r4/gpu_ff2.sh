#!/bin/bash
# round 4: the decoder FF down-projection in one bf16 weight plane too (MTTS_PARITY_FF2_SPLIT=0): parity tests with
# their printed errors, then the bench A/B -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4ff2}; mkdir -p $O; cd $R
MTTS_PARITY_FF2_SPLIT=0 timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_longform_gpu.py -q -s --timeout 300 --timeout-method thread > $O/tests_ff2_oneplane.log 2>&1; rc=$?
tail -1 $O/tests_ff2_oneplane.log; grep -E "^.?bf16-parity: |B=32 bf16-parity: |512x4096 bf16-parity: |FAILED" $O/tests_ff2_oneplane.log | head -20
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
for i in 1 2; do
  for S in 1 0; do
    MTTS_PARITY_FF2_SPLIT=$S timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_split$S.$i.json 2>/dev/null || exit $?
    echo "ff2_split=$S run $i: $(python -c "import json; d=json.loads([l for l in open('$O/ab_split$S.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'], d['precision_check']['modes']['parity_policy'])")"
  done
done
