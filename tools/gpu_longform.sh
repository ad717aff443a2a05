#!/bin/bash
# BASELINE config 5 (long-form stress) on one GPU: B=8, Tx=512, Ty=4096 bench line + rocprofv3 kernel
# stats of the same command (alignment vs decoder split).  Usage: bash tools/gpu_longform.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; TAG=${1:-longform}; mkdir -p $O/$TAG; cd $R
ARGS="--batch 8 --tx 512 --ty 4096 --steps 10 --warmup 3 --no-cpu-baseline --no-synth"
timeout -k 10 400 python bench.py $ARGS > $O/$TAG/bench.json 2> $O/$TAG/bench.err; rc=$?
tail -c 1500 $O/$TAG/bench.json; [ $rc -ne 0 ] && { tail -20 $O/$TAG/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG/prof -o run -- python3 $R/bench.py $ARGS > $O/$TAG/prof_bench.json 2> $O/$TAG/prof.err; rc=$?
echo "prof rc=$rc"; exit $rc
