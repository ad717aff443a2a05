#!/bin/bash
# Fused-loss change: model / training / CFM GPU tests, then the default bench line (no CPU leg).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/loss_check; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_training_gpu.py tests/test_decoder_ops_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth > $O/bench.json 2> $O/bench.err; rc=$?
head -c 400 $O/bench.json; exit $rc
