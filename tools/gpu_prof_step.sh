#!/bin/bash
# kernel-trace profile of the default bench (graph bf16) -> gpurun_out/$1/run_kernel_stats.csv
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; NAME=${1:-prof}; mkdir -p $O/$NAME
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$NAME -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/$NAME/bench.json 2> $O/$NAME/err.log; rc=$?
echo "prof rc=$rc"; tail -c 400 $O/$NAME/bench.json; exit $rc
