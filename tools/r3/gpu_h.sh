#!/bin/bash
# full suite (all failures listed), precision budget, step breakdown, bench, PMC family traffic
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3h}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error:|^E  " $O/gpu_tests.log | head -60; exit $rc; }
timeout -k 10 400 python tools/r3/precision_budget.py split split_encfp32 > $O/precision_budget.jsonl 2> $O/precision_budget.err; rc=$?
echo "budget rc=$rc"; python -c "
import json
for l in open('$O/precision_budget.jsonl'):
    d=json.loads(l); print(d['config'], d['batch'], 'full', [round(x,7) for x in d['full']])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -40 $O/step.txt
cd $R && timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], json.dumps(d['precision_check']['modes']))
print('roofline', {k: d['roofline'][k] for k in ('timing','achieved','frac','avg_launch_us','traffic')})
print('extra', json.dumps(d['extra_configs']))"
TAG=${TAG:-r3h}/pmc bash $R/tools/r3/pmc_families.sh
