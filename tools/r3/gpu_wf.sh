#!/bin/bash
# batched wgrads: kernel-variant A/B (two-half workgroups, 64-row steps) + profile of the default
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wf}; mkdir -p $O; cd $R
for rep in 1 2; do for cfg in "1 32" "2 32" "1 64"; do set -- $cfg
  MTTS_WGRAD_HV=$1 MTTS_WGRAD_KB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('hv=$1 kb=$2 rep $rep', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $T $O/trace.csv
python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -32 $O/step.txt
python3 $R/tools/r3/step_phases.py $T | tee $O/phases.txt
