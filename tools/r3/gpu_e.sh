#!/bin/bash
# split-weight cost by kernel (graph-step breakdowns with MTTS_W_SPLIT=0/1), the full bench line (graph-replay
# roofline leg, 32-true and 16x2 extra lines), PMC traffic per family
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3e}; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for v in 0 1; do
  MTTS_W_SPLIT=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ws$v -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof_ws$v.json 2> $O/prof_ws$v.err; rc=$?
  echo "prof ws=$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof_ws$v.err; exit $rc; }
  T=$(find $O/prof_ws$v -name "*kernel_trace.csv" | head -1); python3 $R/tools/step_breakdown.py $T > $O/step_ws$v.txt; head -24 $O/step_ws$v.txt
done
cd $R && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d['precision_check'])
print('roofline', {k: d['roofline'][k] for k in ('timing','achieved','frac','avg_launch_us','graph_launches_per_step','launches_per_step')})
print('wgrad', {k: d['roofline_wgrad'][k] for k in ('timing','achieved','frac','avg_launch_us')})
print('attn', {k: d['roofline_attn'][k] for k in ('timing','achieved','frac','avg_launch_us')})
print('gprof', {k: v for k, v in d['graph_replay_profile'].items() if k != 'top_kernels_us'})
print('extra', d['extra_configs'])"
cd $R && TAG=${TAG:-r3e}/pmc bash tools/r3/pmc_families.sh
