#!/bin/bash
# round 4: the whole GPU suite + smoke, then the interior-chunk MAS measurements (tools/r4/gpu_mas_interior.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${TAG:-r4chk2} SUITE=1 SMOKE=1 BENCH=0 bash tools/r4/gpu_suite.sh || exit $?
TAG=${TAG:-r4chk2}/mas bash tools/r4/gpu_mas_interior.sh
