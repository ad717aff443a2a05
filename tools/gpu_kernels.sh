#!/bin/bash
# GEMM config sweep + wgrad schedule sweep + the op tests that cover them
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 240 python tools/gemm_sweep.py bf16 ${1:-7,8,11,12} > $O/sweep_panel.log 2>&1 || { tail -30 $O/sweep_panel.log; exit 1; }
timeout -k 10 240 python tools/wgrad_sweep.py bf16 > $O/wgrad_sweep_bf16.log 2>&1 || { tail -20 $O/wgrad_sweep_bf16.log; exit 1; }
timeout -k 10 400 python -m pytest tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_model_gpu.py -x -q -m gpu > $O/kern_tests.log 2>&1; rc=$?; tail -3 $O/kern_tests.log; exit $rc
