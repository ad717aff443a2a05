#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decoder_ops_gpu.py > $O/ops_tests.log 2>&1; rc=$?
tail -5 $O/ops_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_sweep.py bf16 ${1:-7,12,38,41,42} > $O/glds_sweep.log 2>&1; rc=$?
exit $rc
