#!/bin/bash
# one GPU call: precision / DP tests + bench (gpu_precision.sh), then the parity and one-plane step profiles
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${TAG:-r4a} bash tools/r4/gpu_precision.sh; rc=$?
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
TAG=${TAG:-r4a}/prof_parity PREC=bf16-parity bash tools/r4/gpu_prof.sh || exit $?
TAG=${TAG:-r4a}/prof_oneplane PREC=bf16-mixed bash tools/r4/gpu_prof.sh || exit $?
exit $rc
