#!/bin/bash
# rocprofv3 kernel trace of bench.py's timed steps ($BENCH_ARGS) -> step breakdown, phases, per-launch list
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5prof}; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 ${BENCH_ARGS} > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -40 $O/step.txt
python3 $R/tools/r3/step_phases.py $T > $O/phases.txt; cat $O/phases.txt
python3 $R/tools/r4/step_launches.py $T > $O/launches.txt
S=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $S $O/rocprof_kernel_stats.csv
cp $T $O/kernel_trace.csv; rm -rf $O/prof
