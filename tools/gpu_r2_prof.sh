#!/bin/bash
# train-only kernel profile (no synthesise) + per-launch GEMM table
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; NAME=${1:-r2prof}; mkdir -p $O/$NAME; cd $R
timeout -k 10 200 python -u tools/step_gemms.py > $O/$NAME/gemms.txt 2>&1 || { tail $O/$NAME/gemms.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$NAME -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --steps 20 --warmup 3 > $O/$NAME/bench.json 2> $O/$NAME/err.log; rc=$?
echo "prof rc=$rc"; exit $rc
