#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (no CPU baseline) -> gpurun_out/$1/prof
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-p}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth > $O/prof_bench.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/prof.err; exit $rc
