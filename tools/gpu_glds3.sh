#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decoder_ops_gpu.py > $O/ops_tests.log 2>&1; rc=$?
tail -5 $O/ops_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/step_gemms.py > $O/step_gemms.log 2>&1; rc=$?; grep -v amdgpu.ids $O/step_gemms.log | head -40; exit $rc
