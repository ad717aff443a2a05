#!/bin/bash
# Train-step-only kernel profile: rocprofv3 kernel trace of bench.py without the synthesise and CPU
# legs (20 timed + 5 warmup graph replays + the eager roofline pass + MAS timing calls).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; TAG=${1:-tprof}; mkdir -p $O/$TAG; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG/prof -o run -- python3 $R/bench.py --no-synth --no-cpu-baseline > $O/$TAG/bench.json 2> $O/$TAG/prof.err; rc=$?
head -c 600 $O/$TAG/bench.json; echo; echo "prof rc=$rc"; exit $rc
