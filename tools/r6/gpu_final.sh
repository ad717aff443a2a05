#!/bin/bash
# round 6 final snapshot: the whole GPU suite, smoke(), the default bench line, a rocprofv3 step profile, the
# long-form config-5 line -> gpurun_out/$TAG (copied to profiles/r06/final/)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6final}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r5/bench_summary.py $O/bench.json > $O/summary.txt; head -3 $O/summary.txt
TAG=${TAG:-r6final}/prof bash tools/r5/gpu_prof.sh > /dev/null || exit 1
head -3 $O/prof/step.txt
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --no-extra --no-cpu-baseline --no-synth > $O/longform_max.json 2> $O/lf1.err || { tail -5 $O/lf1.err; exit 1; }
python -c "import json,sys; s=open(sys.argv[1]).read(); d=json.loads(s[s.index('{'):]); print('longform ms', d['ms_per_step'], json.dumps(d['roofline_mas']['chain_bound']), d['graph_replay_profile']['top_kernels_us'].get('mas_dp_mw_kernel'))" $O/longform_max.json
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --bucketed 4 --no-extra --no-cpu-baseline --no-synth --no-graph-profile > $O/longform_bucketed.json 2> $O/lf2.err || { tail -5 $O/lf2.err; exit 1; }
python -c "import json,sys; s=open(sys.argv[1]).read(); d=json.loads(s[s.index('{'):]); print('longform bucketed ms', d['ms_per_step'])" $O/longform_bucketed.json
