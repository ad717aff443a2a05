#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r2_dp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_dp_gpu.py tests/test_training_gpu.py \
  > $O/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^E  .*Error" $O/tests.log | cut -c1-300 | tail -30
[ $rc -ne 0 ] && exit $rc
MTTS_FORCE_DP=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth > $O/bench_forcedp.json 2> $O/bench_forcedp.err; rc=$?
tail -c 600 $O/bench_forcedp.json; [ $rc -ne 0 ] && { tail -20 $O/bench_forcedp.err; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth > $O/bench.json 2> $O/bench.err; rc=$?
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('N=1 plain', d['value'], d['ms_per_step'], d['precision_check'])"
python -c "import json;d=json.loads(open('$O/bench_forcedp.json').read().strip().splitlines()[-1]);print('N=1 forced DP', d['value'], d['ms_per_step'], d['dp'])"
exit $rc
