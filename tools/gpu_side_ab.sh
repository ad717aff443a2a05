#!/bin/bash
# training tests + in-step A/B of MTTS_SIDE_WGRAD (0/1, twice each, interleaved)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/side; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_training_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|^FAILED|Error" $O/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
  MTTS_SIDE_WGRAD=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/b.json 2>$O/b_$v.err || exit 1
  python -c "import json;r=json.load(open('$O/b.json'));print('SIDE=$v', r['value'], r['ms_per_step'])"
done
