#!/bin/bash
# phase split of the graph step (rocprof kernel trace) + per-shape GEMM table
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3x}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $T $O/trace.csv
python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -3 $O/step.txt
python3 $R/tools/r3/step_phases.py $T | tee $O/phases.txt
cd $R && timeout -k 10 200 python tools/step_gemms.py > $O/gemms.txt 2>&1; rc=$?; head -45 $O/gemms.txt; exit $rc
