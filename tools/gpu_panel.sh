#!/bin/bash
# GEMM schedule check + timing on the GPU box: panel (cfg 8) vs tile configs, decoder op tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 240 python tools/gemm_sweep.py bf16 ${1:-5,7,8,9,10} > $O/sweep_panel.log 2>&1 || { tail -30 $O/sweep_panel.log; exit 1; }
cat $O/sweep_panel.log
timeout -k 10 400 python -m pytest tests/test_decoder_ops_gpu.py -x -q -m gpu > $O/ops_tests.log 2>&1; rc=$?; tail -5 $O/ops_tests.log; exit $rc
