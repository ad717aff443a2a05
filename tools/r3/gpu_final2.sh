#!/bin/bash
# Round-3 (second session) artifacts: full GPU suite, smoke, PMC HBM traffic per kernel family (written into profiles/r03 on the
# box so the bench line reads it), rocprofv3 kernel stats + step breakdown of the bench, the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-final6}; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/gpu_tests.log | head -40; exit $rc; }
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; [ $rc -ne 0 ] && { tail -20 $O/smoke.log; exit $rc; }
TAG=${TAG:-final6}/pmc bash $R/tools/r3/pmc_families.sh > $O/pmc.log 2>&1; rc=$?
tail -3 $O/pmc.log; [ $rc -ne 0 ] && exit $rc
mkdir -p $R/profiles/r03 && cp $O/pmc/profiles/*_traffic.json $R/profiles/r03/
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -32 $O/step.txt
cd $R && timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], json.dumps(d['precision_check']['modes']))
for k in ('roofline','roofline_wgrad','roofline_attn'):
    r=d.get(k) or {}; print(k, {x: r.get(x) for x in ('timing','achieved','frac','avg_launch_us','traffic')})
print('extra', json.dumps(d['extra_configs']))"
