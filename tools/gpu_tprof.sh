#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python tools/torch_prof.py > $O/torch_prof.log 2>&1; rc=$?; tail -3 $O/torch_prof.log; exit $rc
