#!/bin/bash
# round 4: the GPU suite + smoke + one bench line (no extras) on HEAD -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${TAG:-r4chk} SUITE=1 SMOKE=1 BENCH=1 BENCH_ARGS="--no-graph-profile --no-synth --no-cpu-baseline --steps 30" bash tools/r4/gpu_suite.sh
