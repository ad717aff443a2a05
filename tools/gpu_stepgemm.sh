#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 200 python tools/step_gemms.py > $O/step_gemms.log 2>&1; rc=$?; grep -v amdgpu.ids $O/step_gemms.log | head -60; exit $rc
