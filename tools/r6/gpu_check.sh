#!/bin/bash
# round 6 check: the GPU suite, smoke(), the default bench line, and the two-rank shared-GPU rehearsal of the
# N>1 bench path (gloo transport, watchdog + device progress markers) -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6check}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
[ -n "$TESTS_ONLY" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r5/bench_summary.py $O/bench.json > $O/summary.txt; head -5 $O/summary.txt
MTTS_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 6 --warmup 2 --no-synth > $O/bench_shared2.json 2> $O/bench_shared2.err; rc=$?
echo "shared-gpu 2-rank bench rc=$rc"; python -c "import json,sys; s=open(sys.argv[1]).read(); d=json.loads(s[s.index('{'):]); print(json.dumps(d['dp']))" $O/bench_shared2.json || tail -20 $O/bench_shared2.err
exit $rc
