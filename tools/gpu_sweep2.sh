#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python tools/gemm_sweep2.py $1 $2 > $O/sweep2.log 2>&1; rc=$?; tail -3 $O/sweep2.log; exit $rc
