#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (args passed through), csv output under gpurun_out/$1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; NAME=$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$NAME -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $O/$NAME.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -c 300 $O/$NAME.log
