#!/bin/bash
# round 4: the default bench line (+ extras) and the parity-step profile -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${TAG:-r4b} SUITE=${SUITE:-0} SMOKE=${SMOKE:-0} bash tools/r4/gpu_suite.sh || exit $?
TAG=${TAG:-r4b}/prof PREC=${PREC:-bf16-parity} bash tools/r4/gpu_prof.sh
